#!/bin/bash
# GPU-box check: parity tests, bench, rocprofv3 kernel-trace summary.
# Every GPU step runs under its own timeout; a fault/abort/timeout stops the script
# (exit codes >= 124 other than test failures), ordinary test failures do not.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
STEPS=${STEPS:-tests bench prof}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
if [[ " $STEPS " == *" tests "* ]]; then
  echo "== pytest -m gpu"; date
  timeout -k 10 ${TEST_TIMEOUT:-420} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -30 $OUT/pytest_gpu.log; echo "pytest rc=$rc"
  ok $rc || exit $rc
fi
if [[ " $STEPS " == *" bench "* ]]; then
  echo "== bench"; date
  timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; cat $OUT/bench.json; tail -5 $OUT/bench.err; echo "bench rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
if [[ " $STEPS " == *" prof "* ]]; then
  echo "== rocprofv3 kernel trace"; date
  timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
      python bench.py --steps 100 --warmup 10 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof_bench.json 2> $OUT/prof_bench.err
  rc=$?; echo "prof rc=$rc"; find $OUT/prof -name "*stats*" | head
  [ $rc -eq 0 ] || exit $rc
fi
echo "== done"; date
