#!/bin/bash
# A/B of the fused dW+Adam kernel variants (DQNX_DW16_VAR) and the slab plan: in-context kernel
# times from bench.py (no CPU baseline / extras), then a rocprofv3 kernel trace of the default
set -u
OUT=gpurun_out/${TAG:-r2dw16ab}
mkdir -p $OUT
export TMPDIR=/tmp
for B in ${BATCHES:-1024 4096}; do
  for V in ${VARS:-DQNX_DW16_VAR=0 DQNX_DW16_VAR=1 DQNX_DW16_VAR=2 DQNX_DW16_VAR=3 DQNX_DW16_VAR=4 DQNX_DW_ADAM16=0}; do
    tag=${V//=/_}
    env $V timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --batch $B --steps 200 > $OUT/b${B}_$tag.json 2> $OUT/b${B}_$tag.err || exit $?
    python -c "
import json; d=json.load(open('$OUT/b${B}_$tag.json'))
print('B=$B $V: us/step', round(d['ms_per_step']*1e3,2), [(k['kernel'], round(k['avg_us'],2)) for k in d['kernels']])"
  done
done
if [ -n "${PROF:-}" ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
      python bench.py --no-cpu-baseline --no-extras --no-kernel-timing --steps 200 > $OUT/prof.json 2> $OUT/prof.err || exit $?
  find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-8 | head -20
fi
