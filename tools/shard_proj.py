"""configs[3] shard steps on one GPU: rank 0 of world W (global minibatch 4096, 4096/W rows) --
learn_step(GRADS_ONLY) + apply_grads, with the in-launch prefetch and with the sampler launch.
The W-GPU step adds the RCCL all-reduce of the 428 KB gradient."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "multimodal-drl-rmc_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

args = bench.parse.__wrapped__() if hasattr(bench.parse, "__wrapped__") else None
sys.argv = [sys.argv[0]]
args = bench.parse()
spec = bench.make_spec(args)
dev = torch.device("cuda", 0)
out = {}
for W in (1, 2, 4, 8):
    eng = bench.make_engine(args, spec, 4096, W, 0, dev)
    res = {}
    for pf in (True, False):
        def step(pf=pf):
            eng.learn_step(grads_only=True, prefetch=pf)
            eng.apply_grads(soft_update=True)
        for _ in range(20):
            step()
        el = bench.timed_steps(step, 200, None, dev)
        step(False)
        res["prefetch" if pf else "sampler_launch"] = round(el / 200 * 1e6, 2)
    out[f"w{W}_rows{4096 // W}"] = res
    del eng
    torch.cuda.empty_cache()
print(json.dumps(out))
