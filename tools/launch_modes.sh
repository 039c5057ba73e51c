#!/bin/bash
# Graph replay vs eager launches per workload (one learn step per call).
set -u
mkdir -p gpurun_out
run() {  # name, args
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --no-kernel-timing --steps 100 $2 > gpurun_out/lm_$1.json 2> gpurun_out/lm_$1.err || exit $?
  python -c "
import json
d=json.loads(open('gpurun_out/lm_$1.json').read().strip().splitlines()[-1])
print('$1', round(d['value']/1e6,3), 'M tr/s', round(d['ms_per_step']*1e3,2), 'us/step')"
}
run hyb_graph "--net hybrid --batch 256"
run hyb_eager "--net hybrid --batch 256 --no-graphs"
run per_graph "--algo PerDuelingDoubleDQNAgent"
run per_eager "--algo PerDuelingDoubleDQNAgent --no-graphs"
run c5_graph "--algo PerDuelingDoubleDQNAgent --compute bf16 --batch 8192"
run c5_eager "--algo PerDuelingDoubleDQNAgent --compute bf16 --batch 8192 --no-graphs"
run b4096_graph "--batch 4096"
run b4096_eager "--batch 4096 --no-graphs"
run b4096_eager_pf "--batch 4096 --no-graphs --prefetch"
