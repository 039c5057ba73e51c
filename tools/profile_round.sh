#!/bin/bash
# Round profile of one bench workload (BENCH_ARGS), everything written to gpurun_out/profiles/$ROUND_NAME/ (copied into profiles/ by hand):
#   1. PMC traffic passes (FETCH_SIZE / WRITE_SIZE / TCC hit+miss, one group per rocprofv3 run)
#      -> pmc_traffic_<net>_b<B><TAG>.json (also copied to profiles/, where bench.py reads `traffic`)
#   2. the MFMA pass (tools/pmc_groups_mfma.txt) -> mfma_util_<net>_b<B><TAG>.json
#   3. rocprofv3 --kernel-trace --stats of the same bench command -> kernel_stats.csv
#   4. the full bench line (with its CPU baseline unless BENCH_ARGS says otherwise) -> bench.json
# Every GPU step has its own time limit; a fault / timeout ends the script.
set -u
R=${ROUND_NAME:-round}
OUT=gpurun_out/$R
P=gpurun_out/profiles/$R   # merged back by gpurun; copy into profiles/ afterwards
mkdir -p $OUT $P
export TMPDIR=/tmp
NET=${NET:-mlp}; B=${B:-1024}; TAG=${TAG:-}
NAME=${NET}_b${B}${TAG}
rm -rf gpurun_out/pmc
PMC_GROUPS=tools/pmc_traffic_groups.txt bash tools/pmc.sh || exit $?
python tools/pmc_traffic.py gpurun_out/pmc $P/pmc_traffic_$NAME.json > /dev/null || exit $?
cp $P/pmc_traffic_$NAME.json profiles/pmc_traffic_$NAME.json
rm -rf gpurun_out/pmc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-extras ${BENCH_ARGS:-} > $OUT/prof_bench.json 2> $OUT/prof_bench.err || exit $?
STATS=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cp "$STATS" $P/kernel_stats_$NAME.csv
PMC_GROUPS=tools/pmc_groups_mfma.txt bash tools/pmc.sh || exit $?
python tools/mfma_util.py gpurun_out/pmc $P/mfma_util_$NAME.json $P/kernel_stats_$NAME.csv > /dev/null || exit $?
rm -rf gpurun_out/pmc
if [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $P/bench_$NAME.json 2> $OUT/bench.err || exit $?
  cat $P/bench_$NAME.json
fi
echo "done $NAME"
