"""Diagnostic: the PER sampler launch (k_per_sample) against the number of samples it draws, in
the GRADS_ONLY step of configs[4]'s engine (bf16, PerDuelingDouble, MLP-284): world 1 at global
batch 1024 / 2048 / 8192, and rank 0 of world 8 at 8192 (the replicated draw).  Decides whether
drawing only a rank's own strata would shorten the DP step."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "multimodal-drl-rmc_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from dqn import _capi as C  # noqa: E402

sys.argv = [sys.argv[0], "--algo", "PerDuelingDoubleDQNAgent", "--compute", "bf16", "--no-cpu-baseline", "--no-extras"]
args = bench.parse()
spec = bench.make_spec(args)
dev = torch.device("cuda:0")
for Bg, W in ((1024, 1), (2048, 1), (8192, 1), (8192, 8)):
    eng = bench.make_engine(args, spec, Bg, W, 0, dev)
    for _ in range(20):
        eng.learn_step(grads_only=True)
        bench.shard_td_exchange(eng)
        eng.apply_grads(soft_update=True)
    torch.cuda.synchronize()
    ks = bench.kernel_times(eng, C.STEP_GRADS_ONLY, count=30, reps=3)
    print(f"Bg {Bg} W {W}:", ", ".join(f"{k[0]} {k[1]:.2f}" for k in ks), flush=True)
    del eng
    torch.cuda.empty_cache()
