#!/bin/bash
# same-box A/B of an implicit-conv knob: bench + FETCH/WRITE PMC per arm (gpurun_out/igab/)
# usage: KNOB=DQNX_CIG_GROUPS VALS="1 0" bash tools/r2_igab.sh
mkdir -p gpurun_out/igab
export TMPDIR=/tmp
for v in ${VALS:-1 0}; do
  env $KNOB=$v timeout -k 10 200 python bench.py --net hybrid84 --batch 256 --steps 10 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/igab/b$v.json 2>/dev/null || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    env $KNOB=$v timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/igab/p${v}_$c -o run -- python bench.py --net hybrid84 --batch 256 --steps 5 --warmup 2 --no-extras --no-cpu-baseline --no-kernel-timing > /dev/null 2>&1 || exit 1
  done
  echo "arm $v done"
done
