#!/bin/bash
# GPU tests, then the round profile of the headline workload and of config 5.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
ROUND_NAME=r01b_mlp bash tools/profile_round.sh > gpurun_out/prof_mlp.log 2>&1 || { echo "profile mlp failed"; tail -5 gpurun_out/prof_mlp.log; exit 1; }
echo mlp profile ok
ROUND_NAME=r01b_c5 B=8192 TAG=_bf16 BENCH_ARGS="--batch 8192 --compute bf16 --algo PerDuelingDoubleDQNAgent --cpu-seconds 10" bash tools/profile_round.sh > gpurun_out/prof_c5.log 2>&1 || { echo "profile c5 failed"; tail -5 gpurun_out/prof_c5.log; exit 1; }
echo c5 profile ok
