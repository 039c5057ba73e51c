#!/bin/bash
# GPU-box quick loop: gpu tests, fused-kernel phase stamps, bench summary.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
if [ -z "${NO_STAMPS:-}" ]; then
  timeout -k 10 100 python tools/stamps_fused.py 1024 2>/dev/null | tail -4 || exit $?
fi
timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
python -c "
import json; d=json.load(open('gpurun_out/bench.json')); print('Mtr/s', round(d['value']/1e6,3), 'us/step', round(d['ms_per_step']*1e3,2), [(k['kernel'], round(k['avg_us'],2)) for k in d['kernels']], 'frac', round(d['roofline']['frac'],3))"
