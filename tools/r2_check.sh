#!/bin/bash
# round-2 GPU check: full GPU suite (no -x: see every failure), then the default bench line
set -u
OUT=gpurun_out/${TAG:-r2b}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -25 $OUT/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
if [ -z "${NO_BENCH:-}" ]; then
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench.err
fi
