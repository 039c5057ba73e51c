#!/bin/bash
# Round-2 closing measurements: full GPU suite, MLP round profile (PMC traffic, bench line with CPU
# baseline, rocprofv3 kernel stats), then the configs[4] line (PER + bf16, B=8192) with its stats.
set -u
mkdir -p gpurun_out
bash tools/r2_round.sh || exit $?
OUT=gpurun_out/${ROUND}_c5
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --algo PerDuelingDoubleDQNAgent --compute bf16 --batch 8192 > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python bench.py --algo PerDuelingDoubleDQNAgent --compute bf16 --batch 8192 --steps 100 --warmup 10 --no-cpu-baseline > /dev/null 2>&1 || exit $?
echo c5 done
