#!/bin/bash
# PER samples per sampling workgroup: parity at each setting, then configs[4] / B=1024 bench lines.
set -u
mkdir -p gpurun_out
for spw in 64 128; do
  DQNX_PER_SPW=$spw timeout -k 10 300 python -u -m pytest tests/test_gpu_per.py -k "sample_matches or np_cache or learn_matches" -x -q --timeout 200 --timeout-method thread > gpurun_out/spw_tests_$spw.log 2>&1
  rc=$?; echo "spw $spw: $(tail -1 gpurun_out/spw_tests_$spw.log)"; [ $rc -eq 0 ] || exit $rc
done
for cfg in c5 b1024; do
  args=""; [ $cfg = c5 ] && args="--compute bf16 --batch 8192"
  for spw in 256 128 64; do
    DQNX_PER_SPW=$spw timeout -k 10 200 python bench.py --algo PerDuelingDoubleDQNAgent --no-cpu-baseline --no-extras $args > gpurun_out/spw_${cfg}_$spw.json 2> gpurun_out/spw_${cfg}_$spw.err || exit $?
    python -c "
import json
d=json.loads(open('gpurun_out/spw_${cfg}_$spw.json').read().strip().splitlines()[-1])
print('$cfg spw=$spw', round(d['value']/1e6,2), 'M tr/s', round(d['ms_per_step']*1e3,2), 'us', [(k['kernel'],round(k['avg_us'],2)) for k in d['kernels'] if k['kernel'].startswith('per')])"
  done
done
