#!/bin/bash
# implicit-conv occupancy / band-size knobs on the (4,84,84) bench (gpurun_out/igk/)
mkdir -p gpurun_out/igk
run() { env "$@" timeout -k 10 200 python bench.py --net hybrid84 --batch 256 --steps 10 --warmup 3 --no-extras --no-cpu-baseline; }
run X=0 > gpurun_out/igk/base.json 2>/dev/null || exit 1
run DQNX_CIG_OCC=1 > gpurun_out/igk/occ1.json 2>/dev/null || exit 1
run DQNX_CIG_LDS_KB=100 > gpurun_out/igk/lds100.json 2>/dev/null || exit 1
run DQNX_CIG_LDS_KB=100 DQNX_CIG_OCC=1 > gpurun_out/igk/lds100occ1.json 2>/dev/null || exit 1
run DQNX_CIG_LDS_KB=30 > gpurun_out/igk/lds30.json 2>/dev/null || exit 1
