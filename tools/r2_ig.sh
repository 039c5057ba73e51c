#!/bin/bash
# implicit-GEMM conv check: hybrid84 parity tests + the (4,84,84) bench line (gpurun_out/ig/)
mkdir -p gpurun_out/ig
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_hybrid.py ${PYTEST_K:--k hybrid84} > gpurun_out/ig/test.log 2>&1
rc=$?; echo "test rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --net hybrid84 --batch 256 --steps 10 --warmup 3 --no-extras --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ig/bench.json 2> gpurun_out/ig/bench.err
rc=$?; echo "bench rc=$rc"; exit $rc
