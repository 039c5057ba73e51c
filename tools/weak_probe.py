"""bench.weak_projection (configs[3] weak: rank 0 of world 8, 4096 rows per rank, the global 32,768-sample
draw) under the current DQNX_* environment (PROBE_W: another world size at 4096 rows per rank): one JSON line."""
import json
import os
import sys

sys.argv = ["bench.py", "--steps", "100", "--warmup", "10"]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402

args = bench.parse()
spec = bench.make_spec(args)
r = bench.weak_projection(args, spec, torch.device("cuda:0"), 91.0, W=int(os.environ.get("PROBE_W", "8")))
print(json.dumps(r))
