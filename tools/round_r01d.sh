#!/bin/bash
# Round checkpoint r01d: GPU tests, configs[1] bench line + rocprof stats, configs[2] (4,84,84) and
# (2,27,5) bench lines with CPU baselines + rocprof stats, acting-path latency.
set -u
OUT=gpurun_out/r01d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench_mlp.json 2> $OUT/bench_mlp.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mlp -o run -- \
    python bench.py --steps 200 --warmup 20 --no-cpu-baseline > /dev/null 2> $OUT/prof_mlp.err || exit $?
timeout -k 10 300 python bench.py --net hybrid84 --batch 256 --steps 20 --warmup 3 > $OUT/bench_hybrid84.json 2> $OUT/bench_hybrid84.err || exit $?
timeout -k 10 300 python bench.py --net hybrid --batch 256 --steps 100 --warmup 10 > $OUT/bench_hybrid.json 2> $OUT/bench_hybrid.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_hybrid84 -o run -- \
    python bench.py --net hybrid84 --batch 256 --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing > /dev/null 2> $OUT/prof_h84.err || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
cat $OUT/bench_mlp.json; echo; cat $OUT/smoke.log
echo done
