#!/bin/bash
# Round-2 closing measurements: full GPU suite (no -x), then the MLP round profile (PMC traffic,
# bench line with CPU baseline, rocprofv3 kernel trace) under ROUND's name.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_${ROUND:-r02c}.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu_${ROUND:-r02c}.log; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
ROUND_NAME=${ROUND:-r02c}_mlp bash tools/profile_round.sh > gpurun_out/prof_mlp.log 2>&1 || { echo "profile mlp failed"; tail -5 gpurun_out/prof_mlp.log; exit 1; }
echo mlp profile ok
