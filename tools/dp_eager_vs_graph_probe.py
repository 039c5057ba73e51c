"""The N > 1 bench's configs[3] weak shard step (rank 0 of a world-8 engine: 4096 rows, the global
32,768-sample draw) with a REAL RCCL all-reduce call in it -- a world-1 nccl process group on one GPU
(the collective's host path and stream hand-offs, not xGMI) -- eager dp_learn_step vs GraphedDPStep
replays.  One JSON line."""
import json
import os
import sys

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
sys.argv = ["bench.py", "--steps", "200", "--warmup", "10"]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import bench  # noqa: E402
from dqn.data_parallel import GraphedDPStep, dp_learn_step  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
args = bench.parse()
spec = bench.make_spec(args)
W = int(os.environ.get("PROBE_W", "8"))   # world size of the engine (4096 rows per rank)
eng = bench.make_engine(args, spec, 4096 * W, W, 0, dev)
out = {"world": W}
for _ in range(10):
    dp_learn_step(eng, soft_update=True, prefetch=True)
el = bench.timed_steps(lambda: dp_learn_step(eng, soft_update=True, prefetch=True), args.steps, dist, dev)
out["eager_us"] = el / args.steps * 1e6
dp_learn_step(eng, soft_update=True)   # consume the pending draw
torch.cuda.synchronize()
for gs in (1, 4, 8):
    g = GraphedDPStep(eng, soft_update=True, bucketed=False, prefetch=True, steps=gs)
    g()
    torch.cuda.synchronize()
    n = args.steps // gs
    el = bench.timed_steps(lambda: g(), n, dist, dev)
    out[f"graphed{gs}_us"] = el / (n * gs) * 1e6
    del g
    torch.cuda.synchronize()
    eng.set_graphs(args.graphs)
    dp_learn_step(eng, soft_update=True)
    torch.cuda.synchronize()
eng.check_device_error()
print(json.dumps(out))
dist.destroy_process_group()
