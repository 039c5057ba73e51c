"""Diagnostic: s_memtime phase stamps of conv 1's first k_micro_dw workgroup (block 0, wave 0;
libdqnx_stamps.so) on the HEAD net (Hybrid-284) learn step."""
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
from dqn.engine import LearnEngine, hybrid_spec  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
CAP = 100_000
spec = hybrid_spec(8, "dueling", micro_chw=(2, 27, 5))
eng = LearnEngine(spec, "PerDuelingDoubleDQNAgent", B, CAP, graphs=False)
eng.load_params(bench.init_params(spec))
bench.fill_ring(eng, CAP, spec.obs_dim, 8, eng.device)
random.seed(1234)
eng.set_rng(0, np.array(random.getstate()[1], dtype=np.uint32))
out = (ctypes.c_int64 * 64)()
names = {25: "maps+borders", 26: "first loads issued", 27: "first store+barriers", 36: "stages 2..", 39: "reduce+write"}
for s_ in range(2):
    for k, nm in enumerate(("next loads issued", "mfma loop", "db", "store+barriers")):
        names[28 + 4 * s_ + k] = f"stage {s_} {nm}"
for step in range(5):
    eng.learn_step(soft_update=True)
    torch.cuda.synchronize()
    C.check(C.lib().dqnx_debug_stamps(eng.h, out, eng.stream()), "stamps")
    s = list(out)
    d = s[24:40]
    seq, prev = [], d[0]
    for j in range(1, 16):
        if d[j] and d[j] >= prev:
            seq.append(f"{names.get(24 + j, 24 + j)} {d[j] - prev}")
            prev = d[j]
    print(f"step {step}: micro_dw conv1 wg0 total {prev - d[0]} cyc: " + ", ".join(seq))
