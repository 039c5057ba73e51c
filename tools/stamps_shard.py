"""Diagnostic: phase stamps of the next-minibatch sampler workgroup inside the forward launch of the
configs[3] shard step (rank 0 of world 8, global 4096, prefetching DP steps; libdqnx_stamps.so)."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("DQNX_LIB", os.path.join(HERE, "..", "multimodal-drl-rmc_amd", "dqn", "_lib", "libdqnx_stamps.so"))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "multimodal-drl-rmc_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from dqn import _capi as C  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
sys.argv = [sys.argv[0]]
args = bench.parse()
spec = bench.make_spec(args)
eng = bench.make_engine(args, spec, 4096, W, 0, torch.device("cuda", 0))
out = (ctypes.c_int64 * 64)()
eng.prefetch_prologue()
for step in range(8):
    eng.learn_step(grads_only=True, prefetch=True)
    eng.apply_grads(soft_update=True)
    torch.cuda.synchronize()
    C.check(C.lib().dqnx_debug_stamps(eng.h, out, eng.stream()), "stamps")
    s = list(out)
    body = ["state+clear", "twists", "insert", "scan", "out+pass"]
    print(f"step {step}: in-forward sampler total {s[15] - s[0]} cyc: "
          + ", ".join(f"{body[j]} {s[j + 1] - s[j]}" for j in range(5)) + f", rest {s[15] - s[5]}"
          + (f" [bitmap pass, {s[13] - 1000} repeats: temper {s[7] - s[2]}, atomics {s[8] - s[7]}, "
             f"repeat inserts {s[9] - s[8]}, barrier {s[10] - s[9]}, probes {s[11] - s[10]}, barrier {s[3] - s[11]}]"
             if 1000 <= s[13] < 2000 else ""))
eng.learn_step(grads_only=True)
eng.apply_grads(soft_update=True)
torch.cuda.synchronize()
