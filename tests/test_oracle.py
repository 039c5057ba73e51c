"""Pin the oracle (CPU restatement) against the reference's golden fixtures and against
the reference's own dependencies (CPython random, numpy RandomState).  CPU only."""
import glob
import os
import random
from collections import deque

import numpy as np
import pytest
import torch

from oracle import ref as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_sampler_matches_cpython_random_sample():
    """pyrandom.c random.sample == CPython random.sample(deque, k) (R:dqn/replay_memory.py:39)."""
    rng = np.random.default_rng(0)
    for trial in range(60):
        k = int(rng.integers(1, 300))
        n = int(rng.integers(k, 40000)) if trial % 3 else int(rng.integers(k, k + 40))
        random.seed(trial)
        st = O.py_state_to_array()
        want = random.sample(deque(range(n)), k)
        got = O.sample_positions(st, n, k)
        assert got.tolist() == want
        assert np.array_equal(st, O.py_state_to_array())


def test_sampler_golden():
    z = np.load(os.path.join(GOLDEN, "sampler.npz"))
    for j in range(int(z["count"])):
        st = z[f"c{j}_state_in"].copy()
        got = O.sample_positions(st, int(z[f"c{j}_n"]), int(z[f"c{j}_k"]))
        assert np.array_equal(got, z[f"c{j}_idx"]), j
        assert np.array_equal(st, z[f"c{j}_state_out"]), j


def test_setsize_branch_boundary():
    assert O.sample_setsize(1024) == 21 + 4 ** 6
    assert O.sample_setsize(4096) == 21 + 4 ** 7
    assert O.sample_setsize(5) == 21


def test_np_uniform_golden_and_numpy():
    z = np.load(os.path.join(GOLDEN, "np_uniform.npz"))
    st = z["state_in"].copy()
    lows = z["lows"]
    got = np.array([O.np_uniform(st, lows[i], lows[i + 1]) for i in range(256)])
    assert np.array_equal(got, z["vals"])
    assert np.array_equal(st, z["state_out"])
    np.random.seed(99)
    st = O.np_state_to_array()
    want = [np.random.uniform(0.5 * i, 0.5 * (i + 1)) for i in range(100)]
    got = [O.np_uniform(st, 0.5 * i, 0.5 * (i + 1)) for i in range(100)]
    assert got == want


def test_sumtree_golden():
    z = np.load(os.path.join(GOLDEN, "sumtree.npz"))
    t = O.SumTree(int(z["cap"]))
    for (kind, a, b), out in zip(z["ops"], z["outs"]):
        if kind == 0:
            t.add(b, None)
            assert (t.max_priority_index, t.min_priority_index) == (int(out[0]), int(out[1]))
            assert t.tree[0] == out[2]
        elif kind == 1:
            t.update(int(a), np.float32(b))
            assert (t.max_priority_index, t.min_priority_index) == (int(out[0]), int(out[1]))
            assert t.tree[0] == out[2]
        else:
            leaf, p, _ = t.get_leaf(b)
            assert leaf == int(out[0]) and p == out[2]
    assert np.array_equal(t.tree, z["tree"])


def _spec_for(z):
    tag = str(z["tag"])
    algo = str(z["algo"])
    head = O.algo_spec_head(algo)
    if tag.startswith("mlp"):
        return O.mlp_spec(int(z["obs_dim"]), 8, head)
    return O.hybrid_spec(8, head)


def _sha(*arrays):
    import hashlib
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def run_oracle_from_fixture(z, threads=1):
    torch.set_num_threads(threads)
    spec = _spec_for(z)
    algo = str(z["algo"])
    seed = int(z["seed"])
    init = O.reference_init(spec, seed)
    assert _sha(*[t.numpy() for t in init.values()]) == str(z["init_sha"])
    L = O.OracleLearner(spec, algo, int(z["batch"]), int(z["buffer"]), seed=seed, params=init)
    data = O.synth_transitions(int(z["n_fill"]), int(z["obs_dim"]), 8, seed=seed + 100)
    assert _sha(*data) == str(z["data_sha"])
    O.fill_replay(L, *data)
    L.py_state = z["py_state_in"].copy()
    L.np_state = z["np_state_in"].copy()
    recs = [L.train_step() for _ in range(int(z["steps"]))]
    return L, recs


GOLDEN_LEARN = sorted(glob.glob(os.path.join(GOLDEN, "learn_*.npz")))


@pytest.mark.parametrize("path", GOLDEN_LEARN, ids=[os.path.basename(p)[6:-4] for p in GOLDEN_LEARN])
def test_oracle_learn_golden(path):
    z = np.load(path)
    L, recs = run_oracle_from_fixture(z)
    for s, r in enumerate(recs):
        assert np.array_equal(r.positions, z["pos"][s]), f"step {s} indices"
        assert abs(r.loss - z["loss"][s]) <= 1e-5 * max(1.0, abs(z["loss"][s])), (s, r.loss, z["loss"][s])
        if "isw" in z:
            np.testing.assert_allclose(r.is_weights, z["isw"][s], rtol=1e-12)
            np.testing.assert_allclose(r.abs_td.reshape(-1), z["absd"][s], atol=1e-5)
    if "py_state_out" in z and not str(z["algo"]).startswith("Per"):
        assert np.array_equal(L.py_state, z["py_state_out"])
    if str(z["algo"]).startswith("Per"):
        assert np.array_equal(L.np_state, z["np_state_out"])
    stride = int(z["stride"])
    keys = [str(k) for k in z["keys"]]
    for i, k in enumerate(keys):
        for nm, d in (("online", L.online), ("target", L.target), ("m", L.m), ("v", L.v)):
            ref = z[f"{nm}_{i}"]
            got = d[k].reshape(-1).numpy()
            if ref.size != got.size:
                got = got[::stride]
            tol = 1e-5 if nm in ("online", "target") else 1e-6
            np.testing.assert_allclose(got, ref, atol=tol, rtol=0, err_msg=f"{nm} {k}")


def test_bf16_emulation_linear_matches_explicit_formula():
    """oracle bf16 mode: y = bf16(x) bf16(W)^T + b; dx = bf16(dy) bf16(W) (or dy W); dW = bf16(dy)^T bf16(x)."""
    g = torch.Generator().manual_seed(0)
    x = torch.randn(7, 37, generator=g, requires_grad=True)
    W = torch.randn(11, 37, generator=g, requires_grad=True)
    b = torch.randn(11, generator=g, requires_grad=True)
    dy = torch.randn(7, 11, generator=g)
    for round_dx in (True, False):
        y = O._Bf16Linear.apply(x, W, b, round_dx)
        bx, bW = O.bf16r(x.detach()), O.bf16r(W.detach())
        assert torch.allclose(y, bx @ bW.t() + b, atol=0, rtol=0)
        gx, gW, gb = torch.autograd.grad(y, (x, W, b), dy)
        want_dx = O.bf16r(dy) @ bW if round_dx else dy @ W.detach()
        assert torch.equal(gx, want_dx)
        assert torch.equal(gW, O.bf16r(dy).t() @ bx)
        assert torch.equal(gb, O.bf16r(dy).sum(0))
    # bf16 rounding is round-to-nearest-even on the 16 dropped bits
    v = torch.tensor([1.0 + 2 ** -8, 1.0 + 3 * 2 ** -8, 1.0 + 2 ** -8 + 2 ** -20])
    assert O.bf16r(v).tolist() == [1.0, 1.0 + 2 ** -6, 1.0 + 2 ** -7]


def test_bf16_oracle_learn_close_to_fp32():
    spec = O.mlp_spec(284, 8, "dueling")
    init = O.reference_init(spec, 3)
    data = O.synth_transitions(600, 284, 8, seed=5)
    recs = []
    for compute in ("fp32", "bf16"):
        lr = O.OracleLearner(spec, "DuelingDoubleDQNAgent", 64, 1000, seed=3, params=init, compute=compute)
        O.fill_replay(lr, *data)
        lr.py_state = O.py_state_to_array(random.Random(9).getstate())
        recs.append(lr.train_step())
    a, b = recs
    assert np.array_equal(a.positions, b.positions)
    qa, qb = a.q_online.numpy(), b.q_online.numpy()
    assert 0 < np.abs(qa - qb).max() <= 2e-2 * np.abs(qa).max()


PER_LONG = sorted(glob.glob(os.path.join(GOLDEN, "learn_mlp284long*_PerDuelingDoubleDQNAgent.npz")))


@pytest.mark.parametrize("path", PER_LONG, ids=[os.path.basename(p)[6:-4] for p in PER_LONG])
def test_oracle_per_long_tree_and_cr_pow(path):
    """The 8-step prioritised runs of the reference (make_golden.py mlp284long1024 / mlp284long8192,
    full SumTree kept): the oracle with this host's numpy power (what the reference computed here)
    reproduces the final tree bit for bit; with the correctly rounded float32 power that libdqnx
    computes (oracle pow_mode "cr"), every step's sampled leaves still equal the reference run's and the
    tree differs only by the rounding of the priorities it carries forward (R:dqn/replay_memory.py:94-98,
    R:dqn/utils/sum_tree.py:15-32)."""
    z = np.load(path)
    assert bool(z["tree_full"])
    L, _ = run_oracle_from_fixture(z)
    assert np.array_equal(L.replay.replay_buffer.tree, z["tree"])
    assert L.replay.replay_buffer.max_priority_index == int(z["tree_max_idx"])
    assert L.replay.replay_buffer.min_priority_index == int(z["tree_min_idx"])
    # the same run with the correctly rounded power
    torch.set_num_threads(1)
    spec, seed = _spec_for(z), int(z["seed"])
    Lc = O.OracleLearner(spec, str(z["algo"]), int(z["batch"]), int(z["buffer"]), seed=seed,
                         params=O.reference_init(spec, seed), per_pow="cr")
    O.fill_replay(Lc, *O.synth_transitions(int(z["n_fill"]), int(z["obs_dim"]), 8, seed=seed + 100))
    Lc.py_state, Lc.np_state = z["py_state_in"].copy(), z["np_state_in"].copy()
    for s in range(int(z["steps"])):
        r = Lc.train_step()
        assert np.array_equal(r.positions, z["pos"][s]), f"cr pow moved a sampled leaf at step {s}"
    assert np.array_equal(Lc.np_state, z["np_state_out"])
    t = Lc.replay.replay_buffer.tree
    np.testing.assert_allclose(t, z["tree"], rtol=1e-4, atol=0)
