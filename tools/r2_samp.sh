#!/bin/bash
# sampler check: sampler + engine parity tests, stamps, bench (no CPU baseline)
set -u
OUT=gpurun_out/${TAG:-r2s}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -q -rf --timeout 200 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python tools/stamps_fused.py 1024 > $OUT/stamps1024.txt 2>&1 || exit $?
timeout -k 10 120 python tools/stamps_fused.py 4096 > $OUT/stamps4096.txt 2>&1 || exit $?
tail -n 3 $OUT/stamps1024.txt $OUT/stamps4096.txt
timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench.err
