#!/bin/bash
# Per-kernel PMC summary of one bench workload: one rocprofv3 --pmc pass per line of PMC_GROUPS
# (tools/pmc_groups_conv.txt by default), then tools/pmc_summary.py filtered on FILTER.
# usage: PMC_GROUPS=... FILTER=k_micro BENCH_ARGS="--net hybrid --batch 256" bash tools/pmc_kernel.sh
set -u
rm -rf gpurun_out/pmc
PMC_GROUPS=${PMC_GROUPS:-tools/pmc_groups_conv.txt} BENCH_ARGS="--steps 20 --warmup 3 ${BENCH_ARGS:-}" bash tools/pmc.sh || exit $?
python tools/pmc_summary.py gpurun_out/pmc "${FILTER:-}" > gpurun_out/pmc_summary_${TAG:-x}.txt || exit $?
cat gpurun_out/pmc_summary_${TAG:-x}.txt
