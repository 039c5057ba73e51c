"""Why does a replayed graph of configs[4] shard steps (PER + bf16, global 8192, rank 0 of world 8) time
at ~3x its eager rate on the host clock while a kernel trace shows the kernels back to back?

Measures, on one GPU: the eager step; then graphs of 1 and 4 steps: the host time spent inside
g.replay() (no sync), the wall time of N replays + sync, and HIP-event GPU time of the same replays.
Prints one JSON line."""
import copy
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "multimodal-drl-rmc_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

algo = sys.argv[1] if len(sys.argv) > 1 else "PerDuelingDoubleDQNAgent"
sys.argv = [sys.argv[0]]
args = bench.parse()
a = copy.copy(args)
a.algo = algo
a.compute = "bf16" if algo.startswith("Per") else "fp32"
spec = bench.make_spec(a)
dev = torch.device("cuda", 0)
Bg = 8192 if algo.startswith("Per") else 4096
eng = bench.make_engine(a, spec, Bg, 8, 0, dev)
out = {"algo": algo, "global_batch": Bg}


def shard_step():
    eng.learn_step(grads_only=True)
    if os.environ.get("C5_TD_EXCHANGE", "1") != "0":
        bench.shard_td_exchange(eng)   # (the |delta| all-gather's output: without it the state degenerates)
    eng.apply_grads(soft_update=True)


for _ in range(10):
    shard_step()
torch.cuda.synchronize()
el = bench.timed_steps(shard_step, 100, None, dev)
out["eager_us"] = el / 100 * 1e6

eng.set_graphs(False)
for gs in (1, 4):
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(gs):
            shard_step()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    n = 100 // gs
    # host time inside replay() alone (the GPU may lag behind)
    t_host = 0.0
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(n):
        t1 = time.perf_counter()
        g.replay()
        t_host += time.perf_counter() - t1
    ev1.record()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t0
    out[f"graph{gs}"] = {"replays": n, "host_us_per_replay": t_host / n * 1e6,
                         "enqueue_us_per_step": t_enq / (n * gs) * 1e6,
                         "wall_us_per_step": t_wall / (n * gs) * 1e6,
                         "gpu_event_us_per_step": ev0.elapsed_time(ev1) * 1e3 / (n * gs)}
    # the same replays with a sync after each (latency of one replay)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        g.replay()
        torch.cuda.synchronize()
    out[f"graph{gs}"]["replay_sync_us"] = (time.perf_counter() - t0) / 10 * 1e6
    del g
# eager again after the graphs: a slowdown that comes with the state the steps reach (e.g. the
# SumTree max / min rescans of the priority tracking) shows here too; one from the graphs does not
torch.cuda.synchronize()
for w in range(3):
    el = bench.timed_steps(shard_step, 100, None, dev)
    out.setdefault("eager_after_us", []).append(el / 100 * 1e6)
# bisection: graphs of the shard step's halves alone (timing only: the state they leave is meaningless)
for part, fn in (("learn_only", lambda: eng.learn_step(grads_only=True)),
                 ("apply_only", lambda: eng.apply_grads(soft_update=True))):
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(50):
        g.replay()
    ev1.record()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        fn()
    e1.record()
    torch.cuda.synchronize()
    out[part] = {"graph_us": ev0.elapsed_time(ev1) * 1e3 / 50, "eager_us": e0.elapsed_time(e1) * 1e3 / 50}
    del g
eng.set_graphs(args.graphs)
eng.check_device_error()
print(json.dumps(out), flush=True)
