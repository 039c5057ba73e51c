"""Diagnose bucketed-vs-plain DP differences: run tests/dp_gpu_worker.py ranks (gloo on one GPU) for the
given (world, algo, mode) combos and print, per layer, how many parameters differ and by how much."""
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-drl-rmc_amd")]
from oracle import ref as O  # noqa: E402


def port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run(world, algo, mode, case="c3"):
    d = tempfile.mkdtemp()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port()))
    ps = [subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "dp_gpu_worker.py"), str(r), str(world), algo, d,
                            "global", case, "fp32", mode], env=env) for r in range(world)]
    for p in ps:
        assert p.wait(timeout=400) == 0
    return [np.load(os.path.join(d, f"rank{r}.npz")) for r in range(world)]


for spec in sys.argv[1:]:
    world, algo, mode = spec.split(":")
    world = int(world)
    ref_mode = mode.replace("bucketed", "plain")
    a, b = run(world, algo, ref_mode), run(world, algo, mode)
    layout = [(n, o, int(np.prod(s))) for n, o, s in O.param_layout(O.mlp_spec(284, 8, O.algo_spec_head(algo)))] \
        if hasattr(O, "param_layout") else None
    for r in (0,):
        for k in ("losses", "positions", "params", "target"):
            x, y = a[r][k], b[r][k]
            if np.array_equal(x, y):
                print(spec, r, k, "equal")
                continue
            bad = np.nonzero(x.reshape(-1) != y.reshape(-1))[0]
            print(spec, r, k, f"{bad.size} differ, first {bad[:8]}, max |d| {np.abs(x.reshape(-1) - y.reshape(-1)).max():.3g}")
