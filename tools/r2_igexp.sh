#!/bin/bash
# timing experiments on the implicit conv kernels (results wrong by design): DQNX_CIG_EXP bits
mkdir -p gpurun_out/igexp
for e in 0 1 2 4 8 3 7 15; do
  DQNX_CIG_EXP=$e timeout -k 10 200 python bench.py --net hybrid84 --batch 256 --steps 10 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/igexp/e$e.json 2> gpurun_out/igexp/e$e.err
  rc=$?; echo "exp $e rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
