#!/bin/bash
# Launch-mode comparison of the one-step-per-call path: graph replay vs eager launches, with and
# without the in-launch prefetch (the inter-graph gap is ~8.5 us per hipGraphLaunch on this stack).
set -u
mkdir -p gpurun_out
for v in ${MODES:-graph eager eager_pf graph_pf}; do
  case $v in graph) extra="";; eager) extra="--no-graphs";; eager_pf) extra="--no-graphs --prefetch";; graph_pf) extra="--prefetch";; eager_c8) extra="--no-graphs --chain 8";; graph_c8) extra="--chain 8";; graph_c32) extra="--chain 32";; eager_c32) extra="--no-graphs --chain 32";; esac
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --no-kernel-timing $extra > gpurun_out/gg_$v.json 2> gpurun_out/gg_$v.err || exit $?
  python -c "
import json
d=json.loads(open('gpurun_out/gg_$v.json').read().strip().splitlines()[-1])
print('$v', round(d['value']/1e6,2), 'M tr/s', round(d['ms_per_step']*1e3,2), 'us/step')"
done
