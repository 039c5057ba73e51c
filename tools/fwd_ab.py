"""A/B of forward routes on one GPU: configs[1] (B=1024, prefetching learning loop) and the configs[3]
world-8 shard step (rank 0: 512 rows of global 4096, GRADS_ONLY + apply, prefetch), per route given as
ENV=VAL[,ENV=VAL...] arguments (route knobs are read when an engine is planned).  Each route's kernel
list with in-context times (dqnx_learn_step_omit differences) is printed too.  One JSON line per route."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "multimodal-drl-rmc_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from dqn import _capi as C  # noqa: E402

routes = sys.argv[1:] or [""]
sys.argv = [sys.argv[0]]
args = bench.parse()
spec = bench.make_spec(args)
dev = torch.device("cuda", 0)
for route in routes:
    env = dict(kv.split("=", 1) for kv in route.split(",") if kv)
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    out = {"route": route or "default"}
    try:
        for name, B, W in (("b1024", 1024, 1), ("w8_512", 4096, 8)):
            eng = bench.make_engine(args, spec, B, W, 0, dev)
            go = W > 1

            def step(pf=True):
                eng.learn_step(grads_only=go, prefetch=pf, soft_update=not go)
                if go:
                    eng.apply_grads(soft_update=True)
            for _ in range(30):
                step()
            best = min(bench.timed_steps(step, 300, None, dev) for _ in range(3))
            step(False)
            flags = (C.STEP_GRADS_ONLY if go else C.STEP_SOFT_UPDATE) | C.STEP_PREFETCH
            ks = bench.kernel_times(eng, flags, count=100, reps=5)
            out[name] = {"us_per_step": round(best / 300 * 1e6, 2),
                         "kernels": {k[0]: round(k[1], 2) for k in ks}}
            eng.check_device_error()
            del eng
            torch.cuda.empty_cache()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    print(json.dumps(out), flush=True)
