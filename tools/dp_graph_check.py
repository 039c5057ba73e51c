"""GPU box, world_size 1 over RCCL: the graph-captured data-parallel step (learn kernels +
all-reduce + Adam in one HIP graph) against eager dp_learn_step calls -- identical weights --
and the host-launch cost of each (ms per step)."""
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "multimodal-drl-rmc_amd")]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from dqn import _capi as C  # noqa: E402
from dqn.data_parallel import GraphedDPStep, dp_learn_step  # noqa: E402
from dqn.engine import LearnEngine, mlp_spec  # noqa: E402

algo = sys.argv[1] if len(sys.argv) > 1 else "DuelingDoubleDQNAgent"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
spec = mlp_spec(284, 8, "dueling")


def make():
    e = LearnEngine(spec, algo, B, 100_000, world_size=1, rank=0, device=dev)
    e.load_params(bench.init_params(spec, 0))
    bench.fill_ring(e, 100_000, 284, 8, dev, seed=0)
    random.seed(1234)
    e.set_rng(C.DQNX_RNG_PY, np.array(random.getstate()[1], dtype=np.uint32))
    np.random.seed(1234)
    st = np.random.get_state()
    e.set_rng(C.DQNX_RNG_NP, np.append(st[1], st[2]).astype(np.uint32))
    return e


N = 200
a = make()
for _ in range(3):
    dp_learn_step(a)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    dp_learn_step(a)
torch.cuda.synchronize()
eager_ms = (time.perf_counter() - t0) / N * 1e3

b = make()
for _ in range(3):
    dp_learn_step(b)
g = GraphedDPStep(b)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    g()
torch.cuda.synchronize()
graph_ms = (time.perf_counter() - t0) / N * 1e3

c = make()
for _ in range(3):
    c.learn_step(soft_update=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    c.learn_step(soft_update=True)
torch.cuda.synchronize()
single_ms = (time.perf_counter() - t0) / N * 1e3
# the prefetching DP step (next global minibatch drawn inside the forward launch), graphed
d = make()
for _ in range(3):
    dp_learn_step(d, prefetch=True)
gp = GraphedDPStep(d, prefetch=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N - 1):
    gp()
torch.cuda.synchronize()
pf_ms = (time.perf_counter() - t0) / (N - 1) * 1e3
dp_learn_step(d)   # consumes the pending draw: N + 3 steps in all, like the others
# ... and 4 prefetching steps per graph replay
e = make()
for _ in range(2):
    dp_learn_step(e, prefetch=True)
g4 = GraphedDPStep(e, prefetch=True, steps=4)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N // 4):
    g4()
torch.cuda.synchronize()
pf4_ms = (time.perf_counter() - t0) / N * 1e3
dp_learn_step(e)   # 2 + N + 1 steps
torch.cuda.synchronize()
torch.cuda.synchronize()
same = torch.equal(a.params, b.params) and torch.equal(a.target_params, b.target_params)
same_single = torch.equal(a.params, c.params)
same_pf = torch.equal(a.params, d.params) and torch.equal(a.target_params, d.target_params)
same_pf4 = torch.equal(a.params, e.params) and torch.equal(a.target_params, e.target_params)
print(f"{algo} B={B}: eager dp step {eager_ms * 1e3:.1f} us, graphed dp step {graph_ms * 1e3:.1f} us, "
      f"graphed prefetching dp step {pf_ms * 1e3:.1f} us (4 per replay: {pf4_ms * 1e3:.1f} us), single-GPU learn step "
      f"{single_ms * 1e3:.1f} us; graphed == eager: {same}; dp == single: {same_single}; prefetch == eager: "
      f"{same_pf and same_pf4}")
dist.destroy_process_group()
assert same and same_single and same_pf and same_pf4
