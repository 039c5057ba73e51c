"""configs[3] shard step on one GPU, captured the way the N>1 bench replays it: rank 0 of world W
(global minibatch 4096), `steps` GRADS_ONLY prefetching learn steps + apply_grads per captured
graph (GraphedDPStep without the collective).  Prints us per shard step for W in argv (default 8).
Run under rocprofv3 --kernel-trace for per-kernel durations and gaps (tools/gap_trace.py)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "multimodal-drl-rmc_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

Ws = [int(x) for x in sys.argv[1:]] or [8]
sys.argv = [sys.argv[0]]
args = bench.parse()
spec = bench.make_spec(args)
dev = torch.device("cuda", 0)
out = {}
for W in Ws:
    eng = bench.make_engine(args, spec, 4096, W, 0, dev)
    for _ in range(10):
        eng.learn_step(grads_only=True)
        eng.apply_grads(soft_update=True)
    per_graph = 4
    eng.set_graphs(False)
    eng.prefetch_prologue()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(per_graph):
            eng.learn_step(grads_only=True, prefetch=True)
            eng.apply_grads(soft_update=True)
    for _ in range(10):
        g.replay()
    n = 100
    el = bench.timed_steps(lambda: g.replay(), n, None, dev)
    out[f"w{W}_rows{4096 // W}"] = round(el / (n * per_graph) * 1e6, 2)
    bench.C.check(bench.C.lib().dqnx_prefetch_stream(eng.h, eng.stream()), "prefetch_stream")
    eng.learn_step(grads_only=True)
    eng.check_device_error()
    del g, eng
    torch.cuda.empty_cache()
print(json.dumps(out))
