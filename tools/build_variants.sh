#!/bin/bash
# Build libdqnx variants with different GEMM tile configs into dqn/_lib/var/ (sweep only).
set -e
cd "$(dirname "$0")/../multimodal-drl-rmc_amd"
mkdir -p dqn/_lib/var
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -w"
SRCS=$(sed -n "s/^SRCS := //p" Makefile)
build() { name=$1; shift; /opt/rocm/bin/hipcc $FLAGS "$@" -x hip $SRCS -o dqn/_lib/var/libdqnx_$name.so & }
rm -f dqn/_lib/var/libdqnx_*.so
while read -r name defs; do
  [ -z "$name" ] && continue
  build $name $defs
done < "${1:-/dev/stdin}"
wait
ls dqn/_lib/var
