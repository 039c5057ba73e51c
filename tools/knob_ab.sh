#!/bin/bash
# Quick A/B of an environment knob on the default bench line: KNOB=name VALUES="a b c".
set -u
mkdir -p gpurun_out
for rep in 1 2; do
for v in $VALUES; do
  env $KNOB=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --no-kernel-timing > gpurun_out/knob_$v.json 2> gpurun_out/knob_$v.err || exit $?
  python -c "
import json
d=json.loads(open('gpurun_out/knob_$v.json').read().strip().splitlines()[-1])
print('$KNOB=$v', round(d['value']/1e6,2), 'M tr/s', round(d['ms_per_step']*1e3,2), 'us')"
done
done
