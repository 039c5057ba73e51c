"""configs[4]'s world-8 shard step (bench.c5_projection) under the current DQNX_* environment:
one JSON line with the shard-step times and kernels (round 6: the PER tracking hosted in the apply's
Adam launch, DQNX_PER_TRACK_APPLY=1, against its own k_per_update launch, =0)."""
import json
import os
import sys

sys.argv = ["bench.py", "--steps", os.environ.get("PROBE_STEPS", "100"), "--warmup", "10"]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402

args = bench.parse()
r = bench.c5_projection(args, torch.device("cuda:0"))
r.pop("one_gpu_roofline", None)
r["env"] = {k: v for k, v in os.environ.items() if k.startswith("DQNX_")}
print(json.dumps(r))
