"""Diagnostic (libdqnx_stamps.so): phase stamps of k_dw_bf16d, bf16 uniform replay, B = argv[1] (8192).
Block 0: start (57), first 4 chunks multiplied (58), K loop done (59), slabs stored (60); over all
workgroups: the last end (61) and the workgroup count (62).  Cycles of s_memtime."""
import ctypes
import os
import random
import sys

os.environ.setdefault("DQNX_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                "multimodal-drl-rmc_amd", "dqn", "_lib", "libdqnx_stamps.so"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multimodal-drl-rmc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dqn import _capi as C  # noqa: E402
from dqn.engine import LearnEngine, mlp_spec  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
spec = mlp_spec(284, 8, "dueling")
eng = LearnEngine(spec, "DuelingDoubleDQNAgent", B, 100_000, graphs=False, compute_dtype="bf16")
eng.load_params(bench.init_params(spec))
bench.fill_ring(eng, 100_000, 284, 8, eng.device)
random.seed(1234)
eng.set_rng(0, np.array(random.getstate()[1], dtype=np.uint32))
out = (ctypes.c_int64 * 64)()
for step in range(8):
    eng.learn_step(soft_update=True)
    torch.cuda.synchronize()
    C.check(C.lib().dqnx_debug_stamps(eng.h, out, eng.stream()), "stamps")
    s = list(out)
    t0 = s[57]
    print(f"step {step}: block0 first-4-chunks {s[58] - t0} loop {s[59] - t0} stored {s[60] - t0}; last end {s[61] - t0} "
          f"cycles after block 0's start; workgroups {s[62]}", flush=True)
