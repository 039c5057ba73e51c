#!/usr/bin/env python3
"""`.pack` checkpoint interop in both directions against the REFERENCE's own Network.save / load
(R:dqn/network.py:27-47, through its msgpack-numpy hooks R:dqn/utils/msgpack_numpy.py:74-130).
Build container only: the reference is imported read-only with make_golden.py's recipe
(SURVEY.md §8(c)); nothing of it is copied.  tests/test_pack_interop.py drives the three roles in
separate processes, because the drop-in package and the reference are both named `dqn`:

    pack_interop.py ours-save DIR   drop-in networks (dqn.network) -> DIR/ours_<case>.pack + .npz
    pack_interop.py ref         DIR   reference networks .load(ours_<case>.pack), compare bit for bit;
                                      then the reference saves DIR/ref_<case>.pack + .npz
    pack_interop.py ours-load DIR   drop-in networks .load(ref_<case>.pack), compare bit for bit

Cases: the MLP of R:env/custom_env/macro with lane/dqn_config.py:58-104 at D = 284 (dueling head)
and D = 14 (linear head), and the HEAD TwoStreamHybridNetwork of R:env/dqn_config.py:148-193
(dueling).  Each role prints one "ok <role> <case> ..." line per case."""
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
CASES = (("mlp284_dueling", 284, "dueling", "mlp"), ("mlp14_linear", 14, "linear", "mlp"),
         ("hybrid284_dueling", 284, "dueling", "hybrid"))
META = {"ours": (2_100_000, 23_332, np.float64(-7.25), 90.0), "ref": (12345, 67, np.float64(3.5), 88.0)}


def _perturb(net, seed):
    """Weights away from the default init (every entry a distinct fp32 value)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in net.parameters():
            p.add_(torch.randn(p.shape, generator=g) * 1e-3)


def _state(net):
    return {k: v.detach().cpu().numpy() for k, v in net.state_dict().items()}


def _compare(net, expect_npz, case, role):
    want = np.load(expect_npz)   # (allow_pickle stays False: the file is our own plain arrays)
    got = _state(net)
    assert sorted(got) == sorted(want.files), (case, sorted(got), want.files)
    for k in want.files:
        assert got[k].dtype == want[k].dtype == np.float32 and got[k].shape == want[k].shape, (case, k)
        assert np.array_equal(got[k].view(np.uint32), want[k].view(np.uint32)), (case, k)
    print(f"ok {role} {case}: {len(want.files)} tensors bit-identical", flush=True)


def ours(role, out):
    sys.path[:0] = [os.path.join(REPO, "multimodal-drl-rmc_amd"), os.path.join(REPO, "tests")]
    from dqn import Networks
    from refnets import Box, hybrid_network_config, mlp_network_config
    for i, (case, d, head, kind) in enumerate(CASES):
        cls = Networks.DuelingDeepQNetwork if head == "dueling" else Networks.DeepQNetwork
        conf = mlp_network_config if kind == "mlp" else hybrid_network_config
        torch.manual_seed(100 + i)
        net = cls(torch.device("cpu"), 1e-4, conf, Box(d), 8)
        if role == "ours-save":
            _perturb(net, 200 + i)
            net.save(os.path.join(out, f"ours_{case}.pack"), *META["ours"])
            np.savez(os.path.join(out, f"ours_{case}.npz"), **_state(net))
            print(f"ok ours-save {case}", flush=True)
        else:
            meta = net.load(os.path.join(out, f"ref_{case}.pack"))
            assert tuple(meta) == META["ref"], (case, meta)
            _compare(net, os.path.join(out, f"ref_{case}.npz"), case, role)


def ref(out):
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import importlib

    import make_golden as G   # the import recipe: stubs + bypassed package __init__s
    _agent, _replay, _sumtree, cfg, mlp_cfg = G.load_reference()
    rnet = importlib.import_module("dqn.network")
    for i, (case, d, head, kind) in enumerate(CASES):
        cls = rnet.DuelingDeepQNetwork if head == "dueling" else rnet.DeepQNetwork
        conf = mlp_cfg.network_config if kind == "mlp" else cfg.network_config
        torch.manual_seed(300 + i)
        net = cls(torch.device("cpu"), 1e-4, conf, G.Box(d), 8)
        meta = net.load(os.path.join(out, f"ours_{case}.pack"))
        assert tuple(meta) == META["ours"], (case, meta)
        _compare(net, os.path.join(out, f"ours_{case}.npz"), case, "ref-load")
        _perturb(net, 400 + i)
        net.save(os.path.join(out, f"ref_{case}.pack"), *META["ref"])
        np.savez(os.path.join(out, f"ref_{case}.npz"), **_state(net))
        print(f"ok ref-save {case}", flush=True)


if __name__ == "__main__":
    role, out = sys.argv[1], sys.argv[2]
    if role == "ref":
        ref(out)
    else:
        ours(role, out)
