"""Diagnostic: s_memtime phase stamps (block 0, thread 0) of the PER kernels (libdqnx_stamps.so).
k_per_sample: 0 start, 1 top/MT loaded, 2 words + beta, 3 descents done.
k_per_update (last chunk of the step): 56 start, 57 items loaded, 59 max/min tracking, 61 end.
The tracking workgroup hosted by the gradient launch (any block): 48 start, 49 first items loaded,
50 tracking done; its prop workgroups: 51 hand-off seen, 52 prop done.
Usage: stamps_per.py [batch] [fp32|bf16]"""
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("DQNX_LIB", os.path.join(HERE, "..", "multimodal-drl-rmc_amd", "dqn", "_lib", "libdqnx_stamps.so"))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "multimodal-drl-rmc_amd"))
import ctypes  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dqn import _capi as C  # noqa: E402
from dqn.engine import LearnEngine, mlp_spec  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
cap = 1_000_000
spec = mlp_spec(284, 8, "dueling")
comp = sys.argv[2] if len(sys.argv) > 2 else "fp32"
eng = LearnEngine(spec, "PerDuelingDoubleDQNAgent", B, cap, graphs=False, compute_dtype=comp)
eng.load_params(bench.init_params(spec))
bench.fill_ring(eng, cap, 284, 8, eng.device)
np.random.seed(1234)
st = np.random.get_state()
eng.set_rng(C.DQNX_RNG_NP, np.append(st[1], st[2]).astype(np.uint32))
out = (ctypes.c_int64 * 64)()
for step in range(5):
    eng.learn_step(soft_update=True)
    torch.cuda.synchronize()
    C.check(C.lib().dqnx_debug_stamps(eng.h, out, eng.stream()), "stamps")
    s = list(out)
    ps = [s[j + 1] - s[j] for j in range(3)]
    pu = [s[57] - s[56], s[59] - s[57], s[61] - s[59]]
    print(f"step {step}: per_sample cyc {ps} total {s[3] - s[0]}; per_update cyc {pu} total {s[61] - s[56]}")
    tr = [s[48] - s[56], s[49] - s[48], s[50] - s[49], s[51] - s[50], s[52] - s[51]]
    print(f"  in-launch tracking: start-after-56 / items / tracking / hand-off / prop cyc {tr}")
