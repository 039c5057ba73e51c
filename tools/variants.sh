#!/bin/bash
# Bench variants on the GPU box: one bench line per variant, env knobs from a file.
#   VARIANTS=file OUT=gpurun_out/<dir> BENCH_ARGS="..." bash tools/variants.sh
# Each non-empty line of the file: <name> [VAR=value ...].  Writes <OUT>/<name>.json (the bench line)
# and appends "<name> ms_per_step kernels" to <OUT>/summary.txt.  Every run has its own time limit;
# a failure (fault, abort, time limit) ends the script.
set -u
OUT=${OUT:-gpurun_out/variants}
mkdir -p $OUT
while read -r name envs; do
  [ -z "$name" ] && continue
  case "$name" in \#*) continue ;; esac
  env $envs timeout -k 10 150 python bench.py --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline --no-extras \
      ${BENCH_ARGS:-} > $OUT/$name.json 2> $OUT/$name.err || { echo "FAILED $name rc=$?" >> $OUT/summary.txt; exit 1; }
  python - "$name" "$OUT/$name.json" >> $OUT/summary.txt <<'EOF'
import json, sys
d = json.load(open(sys.argv[2]))
ks = " ".join(f"{k['kernel']}={k['avg_us']:.2f}" for k in d.get("kernels", []))
print(f"{sys.argv[1]:24s} {d['ms_per_step'] * 1e3:7.2f} us  {d['value'] / 1e6:7.2f} M/s  {ks}")
EOF
  tail -1 $OUT/summary.txt
done < ${VARIANTS:?}
