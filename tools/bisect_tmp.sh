set -u
B="python bench.py --steps 20 --warmup 5 --no-kernel-timing --no-cpu-baseline"
echo "== eager, seam"; timeout -k 10 120 $B --no-graphs 2>gpurun_out/b1.err | cut -c1-200 && \
echo "== graphs, no seam"; DQNX_DW_SEAM=0 timeout -k 10 120 $B 2>gpurun_out/b2.err | cut -c1-200 && \
echo "== graphs, seam, plan0"; DQNX_BWD_PLAN=0 timeout -k 10 120 $B 2>gpurun_out/b3.err | cut -c1-200 && \
echo "== graphs, seam"; timeout -k 10 120 $B 2>gpurun_out/b4.err | cut -c1-200
echo "rc=$?"
