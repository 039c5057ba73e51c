"""bench.dropin_loop (the train.py drop-in loop, idle choose_actions) under the current DQNX_*
environment: one JSON line."""
import json
import os
import sys

sys.argv = ["bench.py"]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402

args = bench.parse()
r = bench.dropin_loop(args, torch.device("cuda:0"))
print(json.dumps({k: r[k] for k in ("us_per_iteration", "choose_actions_idle_us", "phases_us")}))
