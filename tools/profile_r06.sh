#!/bin/bash
# Round-6 profiles of the bench workloads named as arguments (mlp_b1024 hybrid_b256 hybrid84_b256
# mlp_b8192_bf16): PMC traffic passes, rocprofv3 --kernel-trace --stats of the same bench command
# bench.py's roofline reads (profiles/r06/kernel_stats_<workload>.csv), the MFMA-busy pass.
# Everything lands under gpurun_out/profiles/r06 (merged back; copied into profiles/ by hand).
set -u
export TMPDIR=/tmp
P=gpurun_out/profiles/r06
mkdir -p $P
for W in "$@"; do
  case $W in
    mlp_b1024) ARGS="" ;;
    hybrid_b256) ARGS="--net hybrid --batch 256" ;;
    hybrid84_b256) ARGS="--net hybrid84 --batch 256" ;;
    mlp_b8192_bf16) ARGS="--algo PerDuelingDoubleDQNAgent --compute bf16 --batch 8192" ;;
    *) echo "unknown workload $W"; exit 2 ;;
  esac
  rm -rf gpurun_out/pmc
  BENCH_ARGS="$ARGS" PMC_GROUPS=tools/pmc_traffic_groups.txt bash tools/pmc.sh || exit $?
  python tools/pmc_traffic.py gpurun_out/pmc $P/pmc_traffic_$W.json > /dev/null || exit $?
  rm -rf gpurun_out/pmc gpurun_out/r06prof_$W
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06prof_$W -o run -- \
      python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-extras $ARGS > $P/prof_bench_$W.json 2> $P/prof_bench_$W.err || exit $?
  STATS=$(find gpurun_out/r06prof_$W -name "*kernel_stats.csv" | head -1)
  cp "$STATS" $P/kernel_stats_$W.csv || exit 1
  rm -rf gpurun_out/r06prof_$W
  BENCH_ARGS="$ARGS" PMC_GROUPS=tools/pmc_groups_mfma.txt bash tools/pmc.sh || exit $?
  python tools/mfma_util.py gpurun_out/pmc $P/mfma_util_$W.json $P/kernel_stats_$W.csv > /dev/null || exit $?
  rm -rf gpurun_out/pmc
  echo "done $W"
done
