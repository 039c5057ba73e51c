"""configs[4] shard step (PER + bf16, global 8192, rank 0 of world 8) on one GPU: eager vs replayed
four per captured graph; run under rocprofv3 --kernel-trace to see the launches of each."""
import copy
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "multimodal-drl-rmc_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "both"
sys.argv = [sys.argv[0]]
args = bench.parse()
a = copy.copy(args)
a.algo, a.compute = "PerDuelingDoubleDQNAgent", "bf16"
spec = bench.make_spec(a)
dev = torch.device("cuda", 0)
eng = bench.make_engine(a, spec, 8192, 8, 0, dev)
out = {}


def shard_step():
    eng.learn_step(grads_only=True)
    eng.apply_grads(soft_update=True)


for _ in range(10):
    shard_step()
if mode in ("both", "eager"):
    el = bench.timed_steps(shard_step, 100, None, dev)
    out["eager_us"] = el / 100 * 1e6
if mode in ("both", "graph"):
    el, gs = bench.graphed_shard_steps(eng, a, 100, dev, prefetch=False)
    out["graph_us"] = el / 100 * 1e6
print(json.dumps(out))
