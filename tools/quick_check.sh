#!/bin/bash
# Quick loop: the fused-plan parity tests, then the default bench line (no CPU baseline / extras).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_per.py tests/test_gpu_bf16.py ${QUICK_TESTS:-} -x -q --timeout 200 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -2 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras ${BENCH_ARGS:-} > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err || exit $?
python - <<'PY'
import json
d = json.loads(open("gpurun_out/quick_bench.json").read().strip().splitlines()[-1])
print(round(d["value"] / 1e6, 2), "M tr/s", round(d["ms_per_step"] * 1e3, 2), "us", d["roofline"]["kernel"], round(d["roofline"]["frac"], 3))
print([(k["kernel"], round(k["avg_us"], 2)) for k in d["kernels"]])
PY
