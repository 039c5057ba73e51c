"""Diagnostic (libdqnx_stamps.so): s_memtime phase stamps of the micro-CNN kernels on the HEAD net
(Hybrid-284 (2,27,5), DuelingDouble, uniform replay, B = argv[1] (256)).

k_micro_fwd, first compute workgroup: input staged (41), conv 1 (42), conv 2 (43), conv 3 + F (44);
over all waves: earliest start (45) / latest end (46).  k_micro_dx, workgroup 0: dF staged (48),
level 2 (49), level 1 (50); all waves: 51 / 52.  k_micro_dw conv 1 workgroup 0: slots 24..39."""
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
CAP = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
spec = hybrid_spec(8, "dueling", micro_chw=(2, 27, 5))
eng = LearnEngine(spec, "DuelingDoubleDQNAgent", B, CAP, graphs=False)
eng.load_params(bench.init_params(spec))
bench.fill_ring(eng, CAP, spec.obs_dim, 8, eng.device)
random.seed(1234)
eng.set_rng(0, np.array(random.getstate()[1], dtype=np.uint32))
out = (ctypes.c_int64 * 64)()
M = 1 << 62
for step in range(6):
    eng.learn_step(soft_update=True)
    torch.cuda.synchronize()
    C.check(C.lib().dqnx_debug_stamps(eng.h, out, eng.stream()), "stamps")
    s = list(out)
    f0 = s[40]
    print(f"step {step}: fwd wg: staged {s[41] - f0} conv1 {s[42] - s[41]} conv2 {s[43] - s[42]} conv3 {s[44] - s[43]} "
          f"(total {s[44] - f0})", flush=True)

    print(f"        fwd wave starts {[s[56 + w] - f0 for w in range(4)]}", flush=True)
    print(f"        dense-1 split wg0: GEMM {s[54] - s[53]} slab store {s[55] - s[54]}", flush=True)
    for nm, b in (("conv2", 53), ("conv3", 0)):
        print(f"        dw {nm} wg: maps {s[b + 1] - s[b]} first stage {s[b + 2] - s[b + 1]} stage 0 {s[b + 3] - s[b + 2]} "
              f"rest {s[b + 4] - s[b + 3]} store {s[b + 5] - s[b + 4]} (total {s[b + 5] - s[b]})", flush=True)
    d0 = s[47]
    print(f"        dx wg0: staged {s[48] - d0} level2 {s[49] - s[48]} level1 {s[50] - s[49]} (total {s[50] - d0})", flush=True)
