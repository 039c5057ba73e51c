#!/bin/bash
# Full GPU parity suite on the box: one pytest process, per-test timeout, log under gpurun_out/.
set -u
OUT=${OUT:-gpurun_out/tests}
mkdir -p $OUT
timeout -k 10 ${TEST_TIMEOUT:-1000} python -u -m pytest tests -m gpu -q -rf --timeout 180 --timeout-method thread \
    ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -25 $OUT/pytest_gpu.log
echo "pytest rc=$rc"
exit $rc
