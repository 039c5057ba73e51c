"""configs[3]'s weak shard step (rank 0 of world 8, 4096 rows per rank, global 32,768 draw) replayed as
bench's N > 1 run replays it (GraphedDPStep's --dp-graph-steps shard steps per graph, the collective
left out): one JSON line, for kernel traces of the graphed step.  PROBE_W: world size (4096 rows per
rank); PROBE_PF=0: the draw as its own launch on the compute stream instead of drawn ahead."""
import json
import os
import sys

sys.argv = ["bench.py", "--steps", os.environ.get("PROBE_STEPS", "200"), "--warmup", "10"]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402

args = bench.parse()
spec = bench.make_spec(args)
dev = torch.device("cuda:0")
W = int(os.environ.get("PROBE_W", "8"))
pf = os.environ.get("PROBE_PF", "1") != "0"
eng = bench.make_engine(args, spec, 4096 * W, W, 0, dev)
for _ in range(5):
    eng.learn_step(grads_only=True)
    eng.apply_grads(soft_update=True)
el, gs = bench.graphed_shard_steps(eng, args, args.steps, dev, prefetch=pf)
print(json.dumps({"world": W, "prefetch": pf, "shard_step_us_graphed": el / args.steps * 1e6, "graph_steps": gs,
                  "env": {k: v for k, v in os.environ.items() if k.startswith("DQNX_")}}))
