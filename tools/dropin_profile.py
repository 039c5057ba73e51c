"""Host-side profile of the drop-in train.py loop (bench.dropin_loop's default agent): cProfile over
the timed iterations, top functions by own time.  Diagnostic only."""
import cProfile
import io
import os
import pstats
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "multimodal-drl-rmc_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

sys.argv = [sys.argv[0]]
args = bench.parse()
pr = cProfile.Profile()
orig = bench.time.perf_counter
state = {"on": False}
pr.enable()
bench.dropin_loop(args, torch.device("cuda", 0), iters=300, warmup=20)
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(28)
print(s.getvalue())
