#!/bin/bash
# A/B of sampler variants: in-context kernel times from bench.py (no CPU baseline / extras)
set -u
OUT=gpurun_out/${TAG:-r2ab}
mkdir -p $OUT
timeout -k 10 120 python tools/stamps_fused.py 1024 > $OUT/stamps1024.txt 2>&1 || exit $?
timeout -k 10 120 python tools/stamps_fused.py 4096 > $OUT/stamps4096.txt 2>&1 || exit $?
grep "sampler" $OUT/stamps1024.txt | tail -2; grep "sampler" $OUT/stamps4096.txt | tail -2
for B in 1024 4096; do
  for V in "" "DQNX_NO_MT_CACHE=1" "DQNX_SAMPLER_OLD=1"; do
    env $V timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --batch $B --steps 100 > $OUT/b${B}_${V%%=*}.json 2> $OUT/b${B}_${V%%=*}.err || exit $?
    python -c "
import json,sys; d=json.load(open('$OUT/b${B}_${V%%=*}.json'))
print('B=$B ${V:-default}: us/step', round(d['ms_per_step']*1e3,2), [(k['kernel'], round(k['avg_us'],2)) for k in d['kernels']])"
  done
done
