"""The drop-in agent loop of bench.py (R:train.py:88-108) alone: one JSON line."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "multimodal-drl-rmc_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

sys.argv = [sys.argv[0]]
args = bench.parse()
print(json.dumps(bench.dropin_loop(args, torch.device("cuda", 0))), flush=True)
