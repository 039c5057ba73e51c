#!/bin/bash
# k_dw_adam16 16 x 16 vs 32 x 16 tiles: parity, then bench lines of both (twice, interleaved).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -k "dw16_row_pair" -x -q --timeout 120 --timeout-method thread > gpurun_out/dw16_tests.log 2>&1
rc=$?; tail -2 gpurun_out/dw16_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for r in 1 2; do
  DQNX_DW16_R=$r timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras > gpurun_out/dw16_r$r.json 2> gpurun_out/dw16_r$r.err || exit $?
  python -c "
import json
d=json.loads(open('gpurun_out/dw16_r$r.json').read().strip().splitlines()[-1])
print('R=$r', round(d['value']/1e6,2), 'M tr/s', round(d['ms_per_step']*1e3,2), 'us', [(k['kernel'],round(k['avg_us'],2)) for k in d['kernels']])"
done
done
