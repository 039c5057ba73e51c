#!/bin/bash
# Learn-loop launch-mode A/B: bench lines per mode (one learn_step per call, --prefetch, --chain C),
# then kernel traces (median kernel durations and inter-kernel gaps) of each.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
MODES=${MODES:-"seq pf c2 c8"}
for mode in $MODES; do
  case $mode in seq) extra="";; pf) extra="--prefetch";; c*) extra="--chain ${mode#c}";; esac
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --no-kernel-timing $extra ${BENCH_ARGS:-} > gpurun_out/ab_$mode.json 2> gpurun_out/ab_$mode.err || exit $?
  python -c "
import json
d=json.loads(open('gpurun_out/ab_$mode.json').read().strip().splitlines()[-1])
print('$mode', round(d['value']/1e6,2), 'M tr/s', round(d['ms_per_step']*1e3,2), 'us/step')"
done
for mode in $MODES; do
  case $mode in seq) extra="";; pf) extra="--prefetch";; c*) extra="--chain ${mode#c}";; esac
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_tr_$mode -o run -- \
      python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-extras --no-kernel-timing $extra ${BENCH_ARGS:-} > /dev/null 2>&1 || exit $?
  echo "== $mode"; python tools/gap_trace.py $(find gpurun_out/ab_tr_$mode -name "*kernel_trace.csv" | head -1)
done
