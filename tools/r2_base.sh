set -u
mkdir -p gpurun_out/r2a
timeout -k 10 120 python tools/stamps_fused.py 1024 > gpurun_out/r2a/stamps1024.txt 2>&1 && \
timeout -k 10 120 python tools/stamps_fused.py 4096 > gpurun_out/r2a/stamps4096.txt 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --batch 4096 > gpurun_out/r2a/bench4096.json 2> gpurun_out/r2a/bench4096.err && \
timeout -k 10 200 python bench.py --no-cpu-baseline --batch 512 > gpurun_out/r2a/bench512.json 2> gpurun_out/r2a/bench512.err
echo rc=$?
