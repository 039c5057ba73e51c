#!/bin/bash
# Round profile: GPU tests, then the headline workload and config 5 (ROUND env names the dirs).
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
ROUND_NAME=${ROUND:-r01c}_mlp bash tools/profile_round.sh > gpurun_out/prof_mlp.log 2>&1 || { echo "profile mlp failed"; tail -5 gpurun_out/prof_mlp.log; exit 1; }
echo mlp profile ok
ROUND_NAME=${ROUND:-r01c}_c5 B=8192 TAG=_bf16 BENCH_ARGS="--batch 8192 --compute bf16 --algo PerDuelingDoubleDQNAgent --cpu-seconds 10" bash tools/profile_round.sh > gpurun_out/prof_c5.log 2>&1 || { echo "profile c5 failed"; tail -5 gpurun_out/prof_c5.log; exit 1; }
echo c5 profile ok
