#!/bin/bash
# Same-box A/B of two builds of libdqnx (DQNX_LIB): bench.py kernel times, alternating runs
set -u
OUT=gpurun_out/${TAG:-ablib}
mkdir -p $OUT
B=${B:-1024}
for r in 1 2; do
  for L in ${LIBS:-libdqnx_base.so libdqnx.so}; do
    DQNX_LIB=multimodal-drl-rmc_amd/dqn/_lib/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --batch $B --steps 300 > $OUT/$L.$r.json 2> $OUT/$L.$r.err || exit $?
    python -c "
import json; d=json.load(open('$OUT/$L.$r.json'))
print('$L run $r B=$B: us/step', round(d['ms_per_step']*1e3,2), [(k['kernel'], round(k['avg_us'],2)) for k in d['kernels']])"
  done
done
