"""GPU box, world_size 1 over RCCL: a graph capture while ProcessGroupNCCL's watchdog thread still holds
an eager collective's work (a hypothesis for round 4's aborts of test_gpu_graphed_bucketed_dp_step,
DESIGN.md §6 -- ruled out: every mode below survives on MI355X / ROCm 7.0 HIP in torch 2.10).

    python tools/capture_watchdog_check.py [package|global|thread_local|nccl_same|nccl_group2]

1. A spin kernel (torch.cuda._sleep) and then an all-reduce are enqueued on the current stream, so the
   all-reduce's work stays incomplete -- and in the watchdog's list, which it polls every ~100 ms with
   hipEventQuery -- for ~1 s.
2. Meanwhile a graph is captured on another stream and the capture is held open for 0.6 s, so the
   watchdog polls the pending work during the capture (deterministically: the work cannot complete
   before the spin kernel ends).
   * "package" (default): dqn.data_parallel.CAPTURE_MODE, the mode of every capture of the package;
   * "global" / "thread_local": torch.cuda.CUDAGraph.capture_begin(capture_error_mode=...);
   * "nccl_same" / "nccl_group2": global mode with a collective captured as well, on the pending work's
     process group (its NCCL stream joins the capture) / on a second group.
3. "package" then also captures the bucketed DP step of the HEAD net (GraphedDPStep(bucketed=True)) with
   its capture stretched by 0.3 s per bucket, right after eager bucketed steps, and checks that replays
   equal eager steps bit for bit.
Exit 0 and one line "capture ok ..." when the process survives."""
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "multimodal-drl-rmc_amd")]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from dqn.data_parallel import CAPTURE_MODE, GraphedDPStep, dp_learn_step_bucketed  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "package"
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
x = torch.ones(1 << 16, device=dev)
dist.all_reduce(x)   # communicator warm-up
torch.cuda.synchronize()

# 1-2: an incomplete collective in the watchdog's list across a held-open capture
g2 = dist.new_group([0]) if mode == "nccl_group2" else None
if g2 is not None:
    dist.all_reduce(x, group=g2)   # (its communicator warm-up)
    torch.cuda.synchronize()
torch.cuda._sleep(int(2.0e9))   # ~1 s of spinning at the loaded clock
dist.all_reduce(x)
side = torch.cuda.Stream(dev)
y = torch.zeros(1 << 16, device=dev)
g = torch.cuda.CUDAGraph()
t0 = time.perf_counter()
cmode = CAPTURE_MODE if mode == "package" else ("global" if mode.startswith("nccl") else mode)
with torch.cuda.stream(side):   # (torch.cuda.graph would synchronise first and let the work complete)
    g.capture_begin(capture_error_mode=cmode)
    y.add_(1.0)
    if mode.startswith("nccl"):   # a captured collective: the PG's NCCL stream joins the capture
        dist.all_reduce(y, group=g2)
    time.sleep(0.6)
    g.capture_end()
held = time.perf_counter() - t0
torch.cuda.synchronize()
g.replay()
torch.cuda.synchronize()
assert float(y[0]) == 1.0, float(y[0])
msg = f"capture ok ({mode}): held open {held:.2f} s with a pending all-reduce in the watchdog"

if mode == "package":
    import bench  # noqa: E402
    from dqn import _capi as C  # noqa: E402
    from dqn.engine import LearnEngine, hybrid_spec  # noqa: E402
    spec = hybrid_spec(8, "dueling", micro_chw=(2, 27, 5))

    def make():
        e = LearnEngine(spec, "DuelingDoubleDQNAgent", 256, 20_000, world_size=1, rank=0, device=dev)
        e.load_params(bench.init_params(spec, 0))
        bench.fill_ring(e, 20_000, spec.obs_dim, 8, dev, seed=0)
        random.seed(1234)
        e.set_rng(C.DQNX_RNG_PY, np.array(random.getstate()[1], dtype=np.uint32))
        return e

    a, c = make(), make()
    for _ in range(3):
        dp_learn_step_bucketed(a)
        dp_learn_step_bucketed(c)
    orig = c.apply_grads_bucket

    def slow_apply(*args, **kw):   # stretches the capture: the watchdog polls inside it
        time.sleep(0.3)
        return orig(*args, **kw)

    c.apply_grads_bucket = slow_apply
    t0 = time.perf_counter()
    gd = GraphedDPStep(c, bucketed=True)
    cap_s = time.perf_counter() - t0
    c.apply_grads_bucket = orig
    for _ in range(5):
        dp_learn_step_bucketed(a)
        gd()
    torch.cuda.synchronize()
    same = torch.equal(a.params, c.params) and torch.equal(a.target_params, c.target_params)
    assert same, "graphed bucketed step != eager bucketed step"
    msg += f"; bucketed HEAD-net DP step captured over {cap_s:.2f} s, 5 replays == eager"
dist.destroy_process_group()
print(msg, flush=True)
