#!/bin/bash
# XCD-aligned row tiles: parity, then bench lines with and without (interleaved, twice).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -k "xcd_row_mapping" -x -q --timeout 120 --timeout-method thread > gpurun_out/xcd_tests.log 2>&1
rc=$?; tail -1 gpurun_out/xcd_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in 0 1; do
  DQNX_XCD_ROWS=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras > gpurun_out/xcd_$v.json 2> gpurun_out/xcd_$v.err || exit $?
  python -c "
import json
d=json.loads(open('gpurun_out/xcd_$v.json').read().strip().splitlines()[-1])
print('xcd_rows=$v', round(d['value']/1e6,2), 'M tr/s', round(d['ms_per_step']*1e3,2), 'us', [(k['kernel'],round(k['avg_us'],2)) for k in d['kernels']])"
done
done
