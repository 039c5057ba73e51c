#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only alongside) on a short bench.
set -u
OUT=gpurun_out/pmc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1; echo "list rc=$?"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL ${PMC_TIMEOUT:-90} rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
     python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-kernel-timing --no-extras ${BENCH_ARGS:-} > $OUT/p$i.json 2> $OUT/p$i.err
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done < ${PMC_GROUPS:-tools/pmc_groups.txt}
