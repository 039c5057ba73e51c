"""Diagnostic: s_memtime phase stamps of the LDS-bitmap sampler (k_sample_bitmap, csrc/sample_body.hpp)
at configs[3]'s weak-scaling draw (k = 32768 = 8 x 4096, n = 10^6), rank 0 of a world-8 engine.
Needs the stamps build (make -C multimodal-drl-rmc_amd stamps)."""
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

k = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
spec = mlp_spec(284, 8, "dueling")
eng = LearnEngine(spec, "DuelingDoubleDQNAgent", k, 1_000_000, world_size=8, rank=0, graphs=False)
eng.load_params(bench.init_params(spec))
bench.fill_ring(eng, 1_000_000, 284, 8, eng.device)
random.seed(1234)
eng.set_rng(0, np.array(random.getstate()[1], dtype=np.uint32))
out = (ctypes.c_int64 * 64)()
names = ["state+clear", "pass0", "twists(p1)", "cands(p1)", "atomics(p1)", "probe(p1)", "scan(p1)", "emit(p1)"]
for step in range(5):
    eng.learn_step(grads_only=True)
    eng.apply_grads(soft_update=True)
    torch.cuda.synchronize()
    C.check(C.lib().dqnx_debug_stamps(eng.h, out, eng.stream()), "stamps")
    s = list(out)
    ph = ", ".join(f"{names[j]} {s[j] - s[j - 1]}" for j in range(1, 8) if s[j] and s[j - 1])
    print(f"step {step}: total {s[15] - s[0]} cycles, passes {s[14]}: {ph}", flush=True)
