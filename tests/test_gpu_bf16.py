"""GPU parity of the bf16 compute mode (BASELINE config 5: PER + Double/Dueling, bf16 compute).

Two checkers, two tolerances:
  * the oracle in bf16 emulation (oracle/ref.py _Bf16Linear: GEMM operands rounded to bf16,
    fp32 sums) -- the same arithmetic up to summation order, so the engine must agree to
    fp32-accumulation noise plus the occasional one-ulp bf16 rounding flip that noise causes;
  * the reference's own fp32 arithmetic (the plain oracle) -- the error the bf16 mode costs,
    bounded by a stated relative tolerance ("bf16 numerics get a looser
    stated tolerance against the fp32 oracle").
Sampling (CPython MT19937 / numpy legacy uniform + SumTree descent) is not affected by the
compute dtype and stays bit-exact.
"""
import random

import numpy as np
import pytest
import torch

from oracle import ref as O

pytestmark = pytest.mark.gpu

# engine vs bf16-emulating oracle.  Summation order differs (fp32 noise, ~1e-7 here); where
# that noise moves a value across a bf16 rounding boundary, the operand downstream differs by
# one bf16 ulp (2^-8 relative).  So: nearly every element within Q_TIGHT, the rest (flip
# descendants, at most Q_FLIP_FRAC of them) within Q_ATOL.
Q_TIGHT = 2e-6
Q_FLIP_FRAC = 2e-2
Q_ATOL = 1e-3          # Q values, targets
LOSS_RTOL = 1e-4
GRAD_TOL = 2e-3        # max |dg| / max |g| per tensor
W_ATOL = 2e-5          # weights after Adam (one lr = 1e-4 is the size of a sign flip)
# engine vs the reference's fp32 arithmetic: stated bf16 error bound
Q_REL_FP32 = 2e-2      # max |dQ| / max |Q|
GRAD_REL_FP32 = 5e-2   # max |dg| / max |g| per tensor


def _E():
    from dqn import engine as E
    return E


def make_bf16_pair(algo, obs_dim, batch, capacity, n_fill, seed, per=False, graphs=True):
    E = _E()
    head = O.algo_spec_head(algo)
    ospec = O.mlp_spec(obs_dim, 8, head)
    init = O.reference_init(ospec, seed)
    kw = dict(seed=seed, params=init)
    if per:
        kw["per_pow"] = "cr"
    emu = O.OracleLearner(ospec, algo, batch, capacity, compute="bf16", **kw)
    ref = O.OracleLearner(ospec, algo, batch, capacity, **kw)
    data = O.synth_transitions(n_fill, obs_dim, 8, seed=seed + 100)
    O.fill_replay(emu, *data)
    O.fill_replay(ref, *data)
    eng = E.LearnEngine(E.mlp_spec(obs_dim, 8, head), algo, batch, capacity, compute_dtype="bf16", graphs=graphs)
    eng.load_params(init)
    eng.push(*data)
    if per:
        np.random.seed(seed + 11)
        st = O.np_state_to_array()
        emu.np_state, ref.np_state = st.copy(), st.copy()
        eng.set_rng(1, st)
    else:
        random.seed(seed + 7)
        st = O.py_state_to_array()
        emu.py_state, ref.py_state = st.copy(), st.copy()
        eng.set_rng(0, st)
    return emu, ref, eng


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def _close(got, want, what):
    d = np.abs(np.asarray(got, np.float64) - np.asarray(want, np.float64))
    frac = float((d > Q_TIGHT).mean())
    assert d.max() <= Q_ATOL and frac <= Q_FLIP_FRAC, (what, float(d.max()), frac)
    return float(d.max()), frac


def _check_step(eng, rec, rec32, step, cap=None):
    if cap is None:
        idx = eng.batch_idx.cpu().numpy().astype(np.int64)
    else:
        idx = eng.batch_idx.cpu().numpy().astype(np.int64) + cap - 1
    assert np.array_equal(idx, rec.positions), f"step {step}: sampled indices differ"
    q = eng.q.cpu().numpy()
    dq = _close(q[0], rec.q_online.numpy(), "Q(s)")
    _close(q[2], rec.q_target_next.numpy(), "Qtarget(s')")
    if rec.q_online_next is not None:
        _close(q[1], rec.q_online_next.numpy(), "Q(s')")
    _close(eng.td[0].cpu().numpy(), rec.targets.view(-1).numpy(), "y")
    assert abs(eng.loss() - rec.loss) <= LOSS_RTOL * max(1.0, abs(rec.loss))
    g = eng.param_views(eng.grads[:-1])
    worst = {}
    for k, r in rec.grads.items():
        worst[k] = _rel(g[k].cpu().numpy(), r.numpy())
        assert worst[k] <= GRAD_TOL, (k, worst[k])
    print(f"step {step}: vs emu: max|dQ| {dq[0]:.2e} ({dq[1]:.1e} beyond fp32 noise), grad rel {max(worst.values()):.2e}")
    if rec32 is not None:   # bf16 error against the reference's fp32 arithmetic
        assert np.array_equal(rec32.positions, rec.positions)
        qr = _rel(q[0], rec32.q_online.numpy())
        assert qr <= Q_REL_FP32, qr
        gr = max(_rel(g[k].cpu().numpy(), r.numpy()) for k, r in rec32.grads.items())
        assert gr <= GRAD_REL_FP32, gr
        print(f"step {step}: vs fp32 reference: Q rel {qr:.2e}, grad rel {gr:.2e}")


def _compare_weights(emu, eng):
    views = {"online": eng.param_views(eng.params), "target": eng.param_views(eng.target_params)}
    for nm, src in (("online", emu.online), ("target", emu.target)):
        for k, r in src.items():
            d = float((views[nm][k].detach().cpu() - r).abs().max())
            assert d <= W_ATOL, (nm, k, d)


@pytest.mark.parametrize("algo,obs_dim,batch,capacity,n_fill,seed", [
    ("DQNAgent", 14, 32, 500, 300, 3),
    ("DoubleDQNAgent", 284, 100, 700, 650, 8),              # ragged last tile
    ("DuelingDoubleDQNAgent", 284, 1024, 20000, 20000, 7),
    ("DuelingDoubleDQNAgent", 284, 8192, 40000, 40000, 9),  # config 5's batch
])
def test_gpu_bf16_learn_matches_bf16_oracle(algo, obs_dim, batch, capacity, n_fill, seed):
    emu, ref, eng = make_bf16_pair(algo, obs_dim, batch, capacity, n_fill, seed)
    for step in range(3):
        rec = emu.train_step()
        eng.learn_step(soft_update=True)
        torch.cuda.synchronize()
        eng.check_device_error()
        _check_step(eng, rec, None, step)
        _compare_weights(emu, eng)
    assert np.array_equal(eng.get_rng(0), emu.py_state)


@pytest.mark.parametrize("algo,obs_dim,batch,capacity,n_fill,seed", [
    ("DuelingDoubleDQNAgent", 284, 1024, 20000, 20000, 17),
    ("DQNAgent", 284, 256, 3000, 3000, 18),
])
def test_gpu_bf16_error_vs_fp32_reference(algo, obs_dim, batch, capacity, n_fill, seed):
    """One step from identical state: the bf16 engine against the reference's fp32 learn step."""
    emu, ref, eng = make_bf16_pair(algo, obs_dim, batch, capacity, n_fill, seed)
    rec = emu.train_step()
    rec32 = ref.train_step()
    eng.learn_step(soft_update=True)
    torch.cuda.synchronize()
    _check_step(eng, rec, rec32, 0)


@pytest.mark.parametrize("obs_dim,batch,cap,n_fill,seed,steps", [
    (14, 32, 500, 300, 3, 1),
    (284, 1024, 20000, 20000, 5, 1),
    (284, 8192, 40000, 40000, 6, 2),   # configs[4] on one GPU: PER + Dueling Double, bf16, B=8192
])
def test_gpu_bf16_per_learn_matches_bf16_oracle(obs_dim, batch, cap, n_fill, seed, steps):
    """Config 5's algorithm: PER + Dueling Double DQN in bf16 (tree sampling bit-exact).  At
    B=8192 the second step samples from the tree the first step's priorities updated."""
    import copy
    from test_gpu_per import assert_tree_equal
    emu, ref, eng = make_bf16_pair("PerDuelingDoubleDQNAgent", obs_dim, batch, cap, n_fill, seed, per=True)
    for step in range(steps):
        t = emu.replay.replay_buffer
        snap = copy.copy(t)
        snap.tree, snap.data = t.tree.copy(), list(t.data)
        rec = emu.train_step()
        eng.learn_step(soft_update=True)
        torch.cuda.synchronize()
        eng.check_device_error()
        _check_step(eng, rec, None, step, cap=cap)
        np.testing.assert_allclose(eng.is_weights.cpu().numpy(), rec.is_weights.astype(np.float32), rtol=2e-7)
        absd = eng.per_abs_td.cpu().numpy()
        _close(absd, rec.abs_td.reshape(-1), "|delta|")
        _compare_weights(emu, eng)
        # the tree update itself is exact: the oracle's SumTree, updated in order with the
        # ENGINE's |delta| (bf16 moves |delta| within the tolerance above), equals the engine's
        # tree bit for bit; the oracle continues from it so the next step samples the same tree
        emu.replay.replay_buffer = snap
        emu.replay.update_batch_priorities(rec.positions.tolist(), absd.reshape(-1, 1))
        assert_tree_equal(eng, snap, exact=True)
    assert np.array_equal(eng.get_rng(1), emu.np_state)


@pytest.mark.parametrize("mr", ["1", "2", "4"])
def test_gpu_bf16_forward_row_tiles(monkeypatch, mr):
    """bf16 fused forward with 16-, 32- and 64-row workgroups (ragged batch)."""
    monkeypatch.setenv("DQNX_FWD_MR", mr)
    emu, ref, eng = make_bf16_pair("DuelingDoubleDQNAgent", 284, 1000, 20000, 20000, 43)
    for step in range(2):
        rec = emu.train_step()
        eng.learn_step(soft_update=True)
        torch.cuda.synchronize()
        _check_step(eng, rec, None, step)
        _compare_weights(emu, eng)


def test_gpu_bf16_graph_and_eager_identical():
    outs = []
    for graphs in (True, False):
        _, _, eng = make_bf16_pair("DuelingDoubleDQNAgent", 284, 512, 4000, 4000, 11, graphs=graphs)
        for _ in range(3):
            eng.learn_step(soft_update=True)
        torch.cuda.synchronize()
        outs.append(eng.params.clone())
    assert torch.equal(outs[0], outs[1])


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1024, 4096])
def test_gpu_bf16_prefetch_bit_identical(batch):
    """bf16 compute with the in-launch prefetch (the bf16 forward hosts the next step's sampler
    workgroup; the slab plan's Adam pass copies the staged minibatch and the blocked bf16 copies
    are rebuilt by a launch of their own): bitwise equal to sequential steps."""
    _, _, e1 = make_bf16_pair("DuelingDoubleDQNAgent", 284, batch, 3 * batch, 3 * batch, 61, graphs=False)
    _, _, e2 = make_bf16_pair("DuelingDoubleDQNAgent", 284, batch, 3 * batch, 3 * batch, 61, graphs=False)
    for i in range(4):
        e1.learn_step(soft_update=True)
        e2.learn_step(soft_update=True, prefetch=i < 3)
    torch.cuda.synchronize()
    assert torch.equal(e1.params, e2.params) and torch.equal(e1.target_params, e2.target_params)
    assert np.array_equal(e1.get_rng(0), e2.get_rng(0))


@pytest.mark.parametrize("algo,batch,per,mr", [
    ("DuelingDoubleDQNAgent", 1024, False, "1"),      # 32 x 32 tiles, 2 slabs, 16-row forward
    ("DuelingDoubleDQNAgent", 8192, False, None),     # 64 x 64 tiles, 16 slabs of 512 samples
    ("DQNAgent", 4096, False, "2"),                   # linear head, 32-row forward tiles
    ("PerDuelingDoubleDQNAgent", 8192, True, None),   # configs[4]: + the tracking / prop workgroups
])
def test_gpu_bf16_t16_dw_bit_identical(monkeypatch, algo, batch, per, mr):
    """k_dw_bf16d (DQNX_DWB_T=1: operands from the slab-transposed bf16 copies the forward and the head
    kernel write, loaded straight into the MFMA fragments) against k_dw_bf16 (the default: fp32 rows
    rounded and transposed through LDS): the same bf16 operands, the same 32-sample MFMA chunks, the same
    slabs -- weights, Adam state and (PER) tree bitwise equal after three steps."""
    if mr is not None:
        monkeypatch.setenv("DQNX_FWD_MR", mr)
    outs = []
    for t16 in ("0", "1"):
        monkeypatch.setenv("DQNX_DWB_T", t16)
        _, _, eng = make_bf16_pair(algo, 284, batch, 3 * batch, 3 * batch, 71, per=per, graphs=False)
        for _ in range(3):
            eng.learn_step(soft_update=True)
        torch.cuda.synchronize()
        eng.check_device_error()
        outs.append([eng.params.clone(), eng.target_params.clone(), eng.adam_m.clone(), eng.adam_v.clone(),
                     eng.grads.clone()] + ([eng.sumtree.clone()] if per else []))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("algo,batch,per", [("DuelingDoubleDQNAgent", 8192, False), ("PerDuelingDoubleDQNAgent", 8192, True)])
def test_gpu_bf16_xcd_rows_multirow_bit_identical(monkeypatch, algo, batch, per):
    """bf16 at configs[4]'s batch runs 64-row forward tiles; with the XCD row mapping the head kernel's
    16-sample tile t follows its row tile t / 4 onto one XCD (DQNX_XCD_ROWS_MR=0: xcd_remap's order).
    Workgroups only move: weights, Adam moments and the tree are bitwise equal."""
    outs = []
    for on in ("0", "1"):
        monkeypatch.setenv("DQNX_XCD_ROWS_MR", on)
        _, _, eng = make_bf16_pair(algo, 284, batch, 3 * batch, 3 * batch, 73, per=per, graphs=False)
        for _ in range(3):
            eng.learn_step(soft_update=True)
        torch.cuda.synchronize()
        eng.check_device_error()
        outs.append([eng.params.clone(), eng.target_params.clone(), eng.adam_v.clone(), eng.q.clone()] +
                    ([eng.sumtree.clone()] if per else []))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
