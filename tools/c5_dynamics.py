"""configs[4]'s shard step (PER + bf16, global 8192, rank 0 of world 8, or the one-GPU step with
argv[1] == "n1") run eagerly for many steps: per-window step time, to show how the step time moves
with the state the training reaches.  Run under rocprofv3 --kernel-trace to see which kernel moves."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "multimodal-drl-rmc_amd")]
import copy  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "w8"
windows = int(sys.argv[2]) if len(sys.argv) > 2 else 6
sys.argv = [sys.argv[0]]
args = bench.parse()
a = copy.copy(args)
a.algo = "PerDuelingDoubleDQNAgent"
a.compute = "bf16"
spec = bench.make_spec(a)
dev = torch.device("cuda", 0)
world = 1 if mode == "n1" else 8
eng = bench.make_engine(a, spec, 8192, world, 0, dev)


def step():
    if world == 1:
        eng.learn_step(soft_update=True)
    else:
        eng.learn_step(grads_only=True)
        if os.environ.get("C5_TD_EXCHANGE", "1") != "0":
            bench.shard_td_exchange(eng)   # (the |delta| all-gather's output)
        eng.apply_grads(soft_update=True)


out = {"mode": mode, "window_us": []}
for w in range(windows):
    el = bench.timed_steps(step, 100, None, dev)
    out["window_us"].append(round(el / 100 * 1e6, 2))
    print(json.dumps({"window": w, "us": out["window_us"][-1]}), flush=True)
c = eng.ctrl()
out["per_max_idx"], out["per_min_idx"] = int(c.per_max_idx), int(c.per_min_idx)
eng.check_device_error()
print(json.dumps(out), flush=True)
