#!/bin/bash
# GPU-box: PER + bf16 parity tests, PER stamps, config-5 bench lines.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_per.py tests/test_gpu_bf16.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_per.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|PASS|FAIL|Error|assert" gpurun_out/pytest_per.log | tail -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python tools/stamps_per.py 8192 2>&1 | tail -3 || exit $?
for cfg in "per_bf16_8192:--batch 8192 --compute bf16 --algo PerDuelingDoubleDQNAgent" "per_fp32_1024:--batch 1024 --algo PerDuelingDoubleDQNAgent"; do
  name=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 $a > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.err
  rc=$?; echo "bench $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$name.err; exit $rc; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_$name.json')); print('$name', 'Mtr/s', round(d['value']/1e6,3), 'us/step', round(d['ms_per_step']*1e3,2), [(k['kernel'], round(k['avg_us'],2)) for k in d['kernels']], 'frac', round(d['roofline']['frac'],4))"
done
