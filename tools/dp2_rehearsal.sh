#!/bin/bash
# World-2 rehearsal of bench.py's N > 1 path on a one-GPU box: two torchrun ranks share cuda:0
# (DQNX_SINGLE_DEVICE=1) and exchange gradients over gloo (RCCL refuses two ranks on one device).
# Runs the strong line (configs[3], global 4096 = 2048 rows per rank), the `weak` extra (4096 rows per
# rank) and the GRADS_ONLY kernel timing, exactly the code the driver's 8-GPU SCALE run executes
# apart from the backend and the graph capture (gloo collectives are host calls).
set -u
OUT=${OUT:-gpurun_out/dp2}
mkdir -p $OUT
export MASTER_ADDR=127.0.0.1
for extra in "" "--algo PerDuelingDoubleDQNAgent --compute bf16 --global-batch 8192 --no-extras"; do
  tag=$([ -z "$extra" ] && echo mlp || echo c5)
  DQNX_SINGLE_DEVICE=1 DQNX_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2962${#tag} \
      bench.py --gpus 2 --steps ${STEPS:-100} --warmup 10 $extra > $OUT/bench_w2_$tag.json 2> $OUT/bench_w2_$tag.err \
      || { tail -20 $OUT/bench_w2_$tag.err; exit 1; }
  tail -c 1500 $OUT/bench_w2_$tag.json
done
