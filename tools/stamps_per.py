"""Diagnostic: s_memtime phase stamps of the PER step's sampler (k_per_sample block 0: slots 0-3) and
of the in-launch tracking workgroup (slots 48-50) at configs[4]'s shape (libdqnx_stamps.so)."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("DQNX_LIB", os.path.join(HERE, "..", "multimodal-drl-rmc_amd", "dqn", "_lib", "libdqnx_stamps.so"))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "multimodal-drl-rmc_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from dqn import _capi as C  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
sys.argv = [sys.argv[0]]
args = bench.parse()
args.algo, args.compute = "PerDuelingDoubleDQNAgent", "bf16"
spec = bench.make_spec(args)
eng = bench.make_engine(args, spec, B, 1, 0, torch.device("cuda", 0))
out = (ctypes.c_int64 * 64)()
for step in range(8):
    eng.learn_step(soft_update=True)
    torch.cuda.synchronize()
    C.check(C.lib().dqnx_debug_stamps(eng.h, out, eng.stream()), "stamps")
    s = list(out)
    ph = ["tree top + MT state loads", "words (cache / twists) + beta", "descents + IS weights"]
    print(f"step {step}: per_sample block 0 total {s[3] - s[0]} cyc: " + ", ".join(f"{ph[j]} {s[j + 1] - s[j]}" for j in range(3)))
    if s[50] and s[48]:
        print(f"         tracking WG: loads {s[49] - s[48]}, scans/rescans {s[50] - s[49]} cyc")
