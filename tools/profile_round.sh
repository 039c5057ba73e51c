#!/bin/bash
# Round profile of the default bench workload: PMC traffic passes (-> the roofline's `traffic`),
# then the full bench line (with CPU baseline), then a rocprofv3 kernel-trace --stats run.
# Every GPU step has its own time limit; a fault / timeout ends the script.
set -u
OUT=gpurun_out/${ROUND_NAME:-round}
mkdir -p $OUT
export TMPDIR=/tmp
NET=${NET:-mlp}; B=${B:-1024}; TAG=${TAG:-}   # TAG=_bf16 for --compute bf16 (bench.py's file name)
PMC_GROUPS=tools/pmc_traffic_groups.txt bash tools/pmc.sh || exit $?
python tools/pmc_traffic.py gpurun_out/pmc $OUT/pmc_traffic_${NET}_b${B}${TAG}.json > /dev/null || exit $?
cp $OUT/pmc_traffic_${NET}_b${B}${TAG}.json profiles/pmc_traffic_${NET}_b${B}${TAG}.json
rm -rf gpurun_out/pmc
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-extras ${BENCH_ARGS:-} > $OUT/prof_bench.json 2> $OUT/prof_bench.err || exit $?
cat $OUT/bench.json
echo done
