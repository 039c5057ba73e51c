"""GPU box, world_size 1 over RCCL, a two-stream conv net or the MLP: the bucketed data-parallel step
(dqn.data_parallel.dp_learn_step_bucketed: per-layer gradient buckets all-reduced and applied on
a side stream while the backward continues) eager and graph-captured, against the unbucketed DP
step and the single-GPU learn step -- identical weights -- with the time per step of each."""
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "multimodal-drl-rmc_amd")]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29534")
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from dqn import _capi as C  # noqa: E402
from dqn.data_parallel import GraphedDPStep, dp_learn_step, dp_learn_step_bucketed  # noqa: E402
from dqn.engine import LearnEngine, hybrid_spec, mlp_spec  # noqa: E402

net = sys.argv[1] if len(sys.argv) > 1 else "hybrid"
algo = "DuelingDoubleDQNAgent"
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
if net == "mlp":   # the fused plan's two buckets, graphed with the in-launch prefetch
    B, cap = 1024, 20_000
    spec = mlp_spec(284, 8, "dueling")
else:
    chw, B, cap = ((2, 27, 5), 256, 20_000) if net == "hybrid" else ((4, 84, 84), 64, 2_000)
    spec = hybrid_spec(8, "dueling", micro_chw=chw)
PF = net == "mlp"


def make():
    e = LearnEngine(spec, algo, B, cap, world_size=1, rank=0, device=dev)
    e.load_params(bench.init_params(spec, 0))
    bench.fill_ring(e, cap, spec.obs_dim, 8, dev, seed=0)
    random.seed(1234)
    e.set_rng(C.DQNX_RNG_PY, np.array(random.getstate()[1], dtype=np.uint32))
    return e


N = 20 if net == "hybrid84" else 100


def timed(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / N * 1e3


# every engine takes 6 + N steps: graph capture needs 3 eager steps first (communicator warm-up)
a = make()
for _ in range(3):
    dp_learn_step(a)
plain_ms = timed(lambda: dp_learn_step(a))
b = make()
for _ in range(3):
    dp_learn_step_bucketed(b)
buck_ms = timed(lambda: dp_learn_step_bucketed(b))
c = make()
for _ in range(3):
    dp_learn_step_bucketed(c)
g = GraphedDPStep(c, bucketed=True, prefetch=PF)
graph_ms = timed(g)
d = make()
for _ in range(3):
    dp_learn_step(d)
gp = GraphedDPStep(d, prefetch=PF)
graph_plain_ms = timed(gp)
s = make()
for _ in range(3):
    s.learn_step(soft_update=True)
single_ms = timed(lambda: s.learn_step(soft_update=True))
# one more step each (the prefetching graphs' last draw is consumed here)
dp_learn_step(a)
dp_learn_step_bucketed(b)
dp_learn_step_bucketed(c)
dp_learn_step(d)
s.learn_step(soft_update=True)
torch.cuda.synchronize()
eq = lambda x, y: torch.equal(x.params, y.params) and torch.equal(x.target_params, y.target_params)  # noqa: E731
pairs = {"plain==bucketed": eq(a, b), "plain==graphed_bucketed": eq(a, c), "plain==graphed_plain": eq(a, d),
         "plain==single": eq(a, s)}
print(pairs, "max|plain-single|", float((a.params - s.params).abs().max()),
      "max|plain-bucketed|", float((a.params - b.params).abs().max()))
same = all(pairs.values())
print(f"{net} B={B} buckets={len(a.dp_buckets())}: eager plain {plain_ms * 1e3:.1f} us, eager bucketed "
      f"{buck_ms * 1e3:.1f} us, graphed bucketed {graph_ms * 1e3:.1f} us, graphed plain {graph_plain_ms * 1e3:.1f} us, "
      f"single-GPU {single_ms * 1e3:.1f} us; all equal: {same}")
dist.destroy_process_group()
assert same
