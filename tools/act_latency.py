"""Acting-path latency on the GPU: Network.actions through dqnx_act vs the
reference's torch forward (R:dqn/network.py:67-74/110-117) on the same resident weights.

Prints one JSON line: per-call host wall time (obs from host numpy, actions back to a list,
as Agent.choose_actions uses it) for both paths, and the device time per dqnx_act launch
over back-to-back launches on device-resident obs."""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-drl-rmc_amd"), os.path.join(REPO, "tests")]
from dqn import engine as E  # noqa: E402
from dqn.network import DuelingDeepQNetwork  # noqa: E402
from refnets import Box, hybrid_network_config, mlp_network_config  # noqa: E402


def wall(fn, iters):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    out = {}
    for tag, conf in (("mlp284", mlp_network_config), ("two_stream", hybrid_network_config)):
        torch.manual_seed(0)
        net = DuelingDeepQNetwork("cuda:0", 1e-4, conf, Box(284), 8)
        out[tag] = measure(net)
    print(json.dumps(out))


def measure(net):
    out = {}
    for n in (1, 8, 64):
        x = np.random.default_rng(n).random((n, 284), dtype=np.float32)
        xt = torch.from_numpy(x).cuda()

        def torch_path():
            with torch.no_grad():
                return net.advantages(torch.as_tensor(x, dtype=torch.float32).to("cuda:0")).argmax(1).tolist()

        got, want = net.actions(x), torch_path()
        assert sum(a != b for a, b in zip(got, want)) <= max(1, n // 32), (got, want)   # fp32 near-ties only
        spec, flat = net._native_act()
        res = torch.empty(n, dtype=torch.int32, device="cuda")
        scratch, desc = E.act_scratch(spec, n, "cuda"), spec.to_c()

        def launch():
            E.act(spec, flat, xt, scratch=scratch, out=res, desc=desc)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(20):
            launch()
        ev0.record()
        for _ in range(500):
            launch()
        ev1.record()
        torch.cuda.synchronize()
        out[f"n{n}"] = {"actions_native_us": wall(lambda: net.actions(x), 500),
                        "actions_torch_us": wall(torch_path, 500),
                        "act_launch_device_us": ev0.elapsed_time(ev1) * 1e3 / 500}
        del res
    return out


if __name__ == "__main__":
    main()
