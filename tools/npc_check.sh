#!/bin/bash
# numpy MT block cache: parity (cache vs twisting), the PER suite, then PER bench lines with and
# without the cache (B=1024 fp32 and configs[4]: bf16 B=8192).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_per.py -x -q --timeout 200 --timeout-method thread > gpurun_out/npc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/npc_tests.log; [ $rc -eq 0 ] || exit $rc
run() {
  env $2 timeout -k 10 200 python bench.py --algo PerDuelingDoubleDQNAgent --no-cpu-baseline --no-extras $3 > gpurun_out/npc_$1.json 2> gpurun_out/npc_$1.err || exit $?
  python -c "
import json
d=json.loads(open('gpurun_out/npc_$1.json').read().strip().splitlines()[-1])
print('$1', round(d['value']/1e6,2), 'M tr/s', round(d['ms_per_step']*1e3,2), 'us', [(k['kernel'],round(k['avg_us'],2)) for k in d['kernels']])"
}
run b1024_cache "" ""
run b1024_nocache "DQNX_NO_NP_CACHE=1" ""
run c5_cache "" "--compute bf16 --batch 8192"
run c5_nocache "DQNX_NO_NP_CACHE=1" "--compute bf16 --batch 8192"
