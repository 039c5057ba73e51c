#!/bin/bash
# Sampler shapes: parity tests, then the shard-step projections per world size (prefetch vs the
# sampler launch) at configs[3]'s global 4096.
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_bf16.py tests/test_gpu_dp.py -k "prefetch or learn_steps or graphed_dp_step_matches" -x -q --timeout 200 --timeout-method thread > gpurun_out/r2f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2f_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/shard_proj.py > gpurun_out/shard_proj.json 2> gpurun_out/shard_proj.err || { tail -5 gpurun_out/shard_proj.err; exit 1; }
cat gpurun_out/shard_proj.json
