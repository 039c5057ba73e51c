#!/bin/bash
# Forward-hosted prefetch: parity tests, then the default bench and the DP projection.
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_dp.py -k "prefetch or learn_steps or graphed_dp_step_matches" -x -q --timeout 200 --timeout-method thread > gpurun_out/r2e_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2e_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2e_bench.json 2> gpurun_out/r2e_bench.err || exit $?
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r2e_bench.json").read().strip().splitlines()[-1])
print(round(d["value"] / 1e6, 2), "M tr/s", round(d["ms_per_step"] * 1e3, 2), "us", d["roofline"]["kernel"], round(d["roofline"]["frac"], 3))
print([(k["kernel"], round(k["avg_us"], 2)) for k in d["kernels"]])
print("configs3_n1", d["configs3_n1"]["ms_per_step"] * 1e3)
p = d["projection_w8"]
print("w8", {k: v for k, v in p.items() if "us" in k}, [(k["kernel"], round(k["avg_us"], 2)) for k in p["kernels_prefetch"]])
PY
