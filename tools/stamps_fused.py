"""Diagnostic: s_memtime phase stamps (block 0, wave 0) of the fused MLP kernels
(libdqnx_stamps.so).  Prints per-phase cycles of k_mlp_fwd and k_head_bwd."""
import ctypes
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("DQNX_LIB", os.path.join(HERE, "..", "multimodal-drl-rmc_amd", "dqn", "_lib", "libdqnx_stamps.so"))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "multimodal-drl-rmc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dqn import _capi as C  # noqa: E402
from dqn.engine import LearnEngine, mlp_spec  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
compute = sys.argv[2] if len(sys.argv) > 2 else "fp32"   # bf16: the configs[4] forward (uniform replay here)
spec = mlp_spec(284, 8, "dueling")
eng = LearnEngine(spec, "DuelingDoubleDQNAgent", B, 1_000_000, graphs=False, compute_dtype=compute)
eng.load_params(bench.init_params(spec))
bench.fill_ring(eng, 1_000_000, 284, 8, eng.device)
random.seed(1234)
eng.set_rng(0, np.array(random.getstate()[1], dtype=np.uint32))
out = (ctypes.c_int64 * 64)()
FWD = ["prologue+gather issue", "gather wait+barrier", "L1 mma", "L1 epi+bar", "L2 mma", "L2 epi+bar",
       "L3 mma", "L3 epi+bar", "-", "head mma", "head reduce"]
for step in range(6):
    eng.learn_step(soft_update=True)
    torch.cuda.synchronize()
    C.check(C.lib().dqnx_debug_stamps(eng.h, out, eng.stream()), "stamps")
    s = list(out)
    f = s[24:38]
    fw = []
    prev = f[0]
    for j in range(1, 14):
        if f[j]:
            fw.append((j, f[j] - prev))
            prev = f[j]
    h = s[40:56]
    hw = []
    prev = h[0]
    for j in range(1, 16):
        if h[j]:
            hw.append((40 + j, h[j] - prev))
            prev = h[j]
    ph = ["loads+clear", "cache/twist", "seen bits", "contended", "ballots", "scan", "out+cache"]
    if s[15] > s[0] and s[15] - s[0] < 10**7:   # multi-pass body (k below the fast path)
        body = ["state+clear", "twists", "insert", "scan", "out+pass"]
        print(f"step {step}: sampler (multi-pass) total {s[15] - s[0]} cyc: "
              + ", ".join(f"{body[j]} {s[j + 1] - s[j]}" for j in range(5)) + f", end {s[15] - s[5]}"
              + f" (twisted blocks {s[16] // 100}, from the cache {s[16] % 100})")
    print(f"step {step}: sampler total {s[7] - s[0]} cyc (nb {s[8]}, cached {s[9]}): "
          + ", ".join(f"{ph[j]} {s[j + 1] - s[j]}" for j in range(7)))
    print(f"step {step}: fwd total {prev and (max(x for x in f if x) - f[0])} cyc: {fw}")
    print(f"         head_bwd total {max(x for x in h if x) - h[0]} cyc: {hw}")
    d = s[56:61]
    if all(d):
        ph = ["prologue", "K loop", "reduce+barrier", "epilogue"]
        print(f"         dw_adam16 (block 0) total {d[4] - d[0]} cyc: "
              + ", ".join(f"{ph[j]} {d[j + 1] - d[j]}" for j in range(4)))
