"""GPU parity of the two-stream hybrid Q-network learn step (TwoStreamHybridNetwork,
R:env/dqn_config.py:66-193: 3 convs with ELU on the (2,27,5) micro grid, concat with the
14 macro features, dense 1358->512->256, dueling / linear head) against the oracle and
the reference's own golden steps."""
import os
import random

import numpy as np
import pytest
import torch

from oracle import ref as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _E():
    from dqn import engine as E
    return E


def make_hybrid_pair(algo, batch, cap, n_fill, seed, graphs=False, micro_chw=(2, 27, 5)):
    E = _E()
    head = O.algo_spec_head(algo)
    ospec = O.hybrid_spec(8, head, micro_chw=micro_chw)
    init = O.reference_init(ospec, seed)
    oracle = O.OracleLearner(ospec, algo, batch, cap, seed=seed, params=init, per_pow="cr")
    data = O.synth_transitions(n_fill, ospec.obs_dim, 8, seed=seed + 100)
    O.fill_replay(oracle, *data)
    eng = E.LearnEngine(E.hybrid_spec(8, head, micro_chw=micro_chw), algo, batch, cap, graphs=graphs)
    eng.load_params(init)
    eng.push(*data)
    random.seed(seed + 7)
    st = O.py_state_to_array()
    oracle.py_state = st.copy()
    eng.set_rng(0, st)
    np.random.seed(seed + 11)
    nps = O.np_state_to_array()
    oracle.np_state = nps.copy()
    eng.set_rng(1, nps)
    return oracle, eng


@pytest.mark.parametrize("algo,batch,cap,n_fill,seed", [
    ("DuelingDoubleDQNAgent", 32, 500, 300, 3),
    ("DQNAgent", 64, 1000, 700, 4),
    ("DuelingDoubleDQNAgent", 256, 5000, 3000, 5),
    ("PerDuelingDoubleDQNAgent", 64, 1000, 700, 6),
])
def test_gpu_hybrid_learn_matches_oracle(algo, batch, cap, n_fill, seed):
    oracle, eng = make_hybrid_pair(algo, batch, cap, n_fill, seed)
    per = algo.startswith("Per")
    for step in range(3):
        rec = oracle.train_step()
        eng.learn_step(soft_update=True)
        torch.cuda.synchronize()
        eng.check_device_error()
        idx = eng.batch_idx.cpu().numpy().astype(np.int64) + (cap - 1 if per else 0)
        assert np.array_equal(idx, rec.positions), f"step {step}: sampled indices differ"
        q = eng.q.cpu()
        np.testing.assert_allclose(q[0].numpy(), rec.q_online.numpy(), atol=1e-5, rtol=1e-5)
        np.testing.assert_allclose(q[2].numpy(), rec.q_target_next.numpy(), atol=1e-5, rtol=1e-5)
        assert abs(eng.loss() - rec.loss) <= 1e-5 * max(1.0, abs(rec.loss))
        g = eng.param_views(eng.grads[:-1])
        for k, ref in rec.grads.items():
            np.testing.assert_allclose(g[k].cpu().numpy(), ref.numpy(), atol=5e-6, rtol=1e-3, err_msg=k)
        on = eng.param_views(eng.params)
        tg = eng.param_views(eng.target_params)
        for k in oracle.online:
            np.testing.assert_allclose(on[k].cpu().numpy(), oracle.online[k].numpy(), atol=1e-5, rtol=0, err_msg=k)
            np.testing.assert_allclose(tg[k].cpu().numpy(), oracle.target[k].numpy(), atol=1e-5, rtol=0, err_msg=k)


@pytest.mark.parametrize("micro", ["1", "0"])
def test_gpu_hybrid_conv_routes_match_oracle(monkeypatch, micro):
    """The (2,27,5) HEAD net's two conv routes against the oracle: the micro-CNN plan (micro.hip,
    the default: every conv of every stream in one forward launch, the phase-split data gradients
    and the sample-sliced weight gradients in two more) and the per-layer explicit plan
    (DQNX_MICRO_CNN=0: im2col + GEMM, col2im).  PER at a batch that is no multiple of anything."""
    monkeypatch.setenv("DQNX_MICRO_CNN", micro)
    test_gpu_hybrid_learn_matches_oracle("PerDuelingDoubleDQNAgent", 100, 1000, 700, 31)


def test_gpu_hybrid_learn_golden():
    """Against the reference's own hybrid DuelingDouble steps (tests/golden/make_golden.py)."""
    E = _E()
    z = np.load(os.path.join(GOLDEN, "learn_hybrid284_DuelingDoubleDQNAgent.npz"))
    init = O.reference_init(O.hybrid_spec(8, "dueling"), int(z["seed"]))
    eng = E.LearnEngine(E.hybrid_spec(8, "dueling"), str(z["algo"]), int(z["batch"]), int(z["buffer"]))
    eng.load_params(init)
    eng.push(*O.synth_transitions(int(z["n_fill"]), int(z["obs_dim"]), 8, seed=int(z["seed"]) + 100))
    eng.set_rng(0, z["py_state_in"])
    for s in range(int(z["steps"])):
        eng.learn_step(soft_update=True)
        torch.cuda.synchronize()
        assert np.array_equal(eng.batch_idx.cpu().numpy().astype(np.int64), z["pos"][s])
        assert abs(eng.loss() - z["loss"][s]) <= 1e-5 * max(1.0, abs(z["loss"][s]))
    assert np.array_equal(eng.get_rng(0), z["py_state_out"])
    stride = int(z["stride"])
    keys = [str(k) for k in z["keys"]]
    on, tg = eng.param_views(eng.params), eng.param_views(eng.target_params)
    for i, k in enumerate(keys):
        got = on[k].cpu().numpy().reshape(-1)
        ref = z[f"online_{i}"]
        if got.size != ref.size:
            got = got[::stride]
        np.testing.assert_allclose(got, ref, atol=1e-5, rtol=0, err_msg=k)


@pytest.mark.parametrize("batch,fwd_big,conv_ig", [(64, "1", "1"), (128, "1", "1"), (128, "1", "0"), (128, "0", "0"),
                                             (256, "1", "1")])
def test_gpu_hybrid84_learn_matches_oracle(monkeypatch, batch, fwd_big, conv_ig):
    """The stacked (4,84,84) variant (BASELINE configs[2]).  conv_ig=1 (the default): the
    implicit-GEMM convs of conv_ig.hip (forward with F written by the last conv, phase-split data
    gradients, row-group dW slabs) and the 128x128 split-K forward of the 56,462-wide dense layer.
    conv_ig=0: the explicit path -- LDS band im2col (convs 1-2), conv GEMMs, col2im; B=128 takes
    the kernel routes of the B=256 bench: conv 2 and conv 3 (882*B >= 65,536 rows) on the 64x128
    k_conv_dw_big tiles; with DQNX_FWD_BIG=0 the conv dX runs as the split conv_dxs level beside
    the big dW.  Tolerances are those of the (2,27,5) cases, with the
    gradient check scale-relative (the 56,462-term sums differ from torch's CPU order by a few
    ulps of the largest terms).  B=256 is the bench's batch (configs[2]): the default implicit
    path with the split-K count of the 56,462-wide dense layer chosen for 256 rows per GPU."""
    E = _E()
    from parity import assert_grad_close
    monkeypatch.setenv("DQNX_FWD_BIG", fwd_big)
    monkeypatch.setenv("DQNX_CONV_IG", conv_ig)
    algo, seed = "DuelingDoubleDQNAgent", 8
    cap, n_fill = (200, 150) if batch < 256 else (400, 350)
    ospec = O.hybrid_spec(8, "dueling", micro_chw=(4, 84, 84))
    init = O.reference_init(ospec, seed)
    oracle = O.OracleLearner(ospec, algo, batch, cap, seed=seed, params=init)
    data = O.synth_transitions(n_fill, ospec.obs_dim, 8, seed=seed + 100)
    O.fill_replay(oracle, *data)
    eng = E.LearnEngine(E.hybrid_spec(8, "dueling", micro_chw=(4, 84, 84)), algo, batch, cap)
    eng.load_params(init)
    eng.push(*data)
    random.seed(seed + 7)
    st = O.py_state_to_array()
    oracle.py_state = st.copy()
    eng.set_rng(0, st)
    for step in range(2):
        rec = oracle.train_step()
        eng.learn_step(soft_update=True)
        torch.cuda.synchronize()
        eng.check_device_error()
        assert np.array_equal(eng.batch_idx.cpu().numpy().astype(np.int64), rec.positions)
        q = eng.q.cpu()
        np.testing.assert_allclose(q[0].numpy(), rec.q_online.numpy(), atol=1e-5, rtol=1e-5)
        np.testing.assert_allclose(q[2].numpy(), rec.q_target_next.numpy(), atol=1e-5, rtol=1e-5)
        assert abs(eng.loss() - rec.loss) <= 1e-5 * max(1.0, abs(rec.loss))
        g = eng.param_views(eng.grads[:-1])
        for k, ref in rec.grads.items():
            assert_grad_close(g[k].cpu(), ref, k)
        on = eng.param_views(eng.params)
        for k in oracle.online:
            np.testing.assert_allclose(on[k].cpu().numpy(), oracle.online[k].numpy(), atol=1e-5, rtol=0, err_msg=k)


@pytest.mark.parametrize("algo,batch,seed", [("DQNAgent", 32, 21), ("PerDuelingDoubleDQNAgent", 32, 22),
                                             ("DoubleDQNAgent", 48, 23)])
def test_gpu_hybrid84_implicit_convs_all_algorithms(algo, batch, seed):
    """The implicit-GEMM conv path (conv_ig.hip) under every algorithm: two forward streams
    (DQNAgent: online(s), target(s')), the linear head, PER (IS weights through the conv
    backward), a batch that is no multiple of the row tiles."""
    from parity import assert_grad_close
    from test_gpu_engine import compare_state
    cap, n_fill = 200, 150
    oracle, eng = make_hybrid_pair(algo, batch, cap, n_fill, seed, micro_chw=(4, 84, 84))
    per = algo.startswith("Per")
    loose = {k: torch.zeros_like(v, dtype=torch.bool) for k, v in oracle.online.items()}
    for step in range(2):
        rec = oracle.train_step()
        eng.learn_step(soft_update=True)
        torch.cuda.synchronize()
        eng.check_device_error()
        idx = eng.batch_idx.cpu().numpy().astype(np.int64) + (cap - 1 if per else 0)
        assert np.array_equal(idx, rec.positions), f"step {step}: sampled indices differ"
        q = eng.q.cpu()
        np.testing.assert_allclose(q[0].numpy(), rec.q_online.numpy(), atol=1e-5, rtol=1e-5)
        np.testing.assert_allclose(q[2].numpy(), rec.q_target_next.numpy(), atol=1e-5, rtol=1e-5)
        assert abs(eng.loss() - rec.loss) <= 1e-5 * max(1.0, abs(rec.loss))
        g = eng.param_views(eng.grads[:-1])
        for k, ref in rec.grads.items():
            got = g[k].cpu()
            assert_grad_close(got, ref, k)
            loose[k] |= (got - ref).abs() > 1e-3 * ref.abs()
        # weights at 1e-5, except (capped, counted) entries whose gradient differed by > 0.1 %
        # (Adam's lr * g / |g| step, see test_gpu_engine.compare_state)
        compare_state(oracle, eng, loose=loose)


@pytest.mark.parametrize("algo,batch,grads_only", [("DuelingDoubleDQNAgent", 256, False), ("DQNAgent", 100, False),
                                                   ("DuelingDoubleDQNAgent", 256, True)])
def test_gpu_hybrid_inlaunch_prefetch_bit_identical(algo, batch, grads_only):
    """The HEAD net's micro-CNN plan under DQNX_STEP_PREFETCH: k_micro_fwd's block 0 draws step
    t+1's minibatch into the staging slot and the step's last launch (Adam, or the gradient reduce
    of a GRADS_ONLY step) copies it over the compute slot.  Bitwise equal to sequential steps: Q,
    gradients, weights, the sampled indices and the RNG state."""
    o1, e1 = make_hybrid_pair(algo, batch, 3000, 2500, 61)
    o2, e2 = make_hybrid_pair(algo, batch, 3000, 2500, 61)
    for i in range(5):
        e1.learn_step(soft_update=not grads_only, grads_only=grads_only)
        e2.learn_step(soft_update=not grads_only, grads_only=grads_only, prefetch=i < 4)
        if grads_only:
            e1.apply_grads(soft_update=True)
            e2.apply_grads(soft_update=True)
    torch.cuda.synchronize()
    e1.check_device_error()
    e2.check_device_error()
    assert torch.equal(e1.batch_idx, e2.batch_idx)
    assert torch.equal(e1.q, e2.q) and torch.equal(e1.grads, e2.grads)
    assert torch.equal(e1.params, e2.params) and torch.equal(e1.target_params, e2.target_params)
    assert np.array_equal(e1.get_rng(0), e2.get_rng(0))


@pytest.mark.parametrize("algo", ["DuelingDoubleDQNAgent", "PerDuelingDoubleDQNAgent"])
def test_gpu_hybrid_adam_written_conv_copies_bit_identical(algo):
    """Eager micro-CNN steps skip the conv_perm launch while the permuted conv weight copies are
    current: the previous step's Adam pass wrote them next to every updated conv weight (wide slab
    path).  Against an engine replaying graphs (which always launch conv_perm): bitwise equal through
    hard / soft updates, a direct parameter write (+ params_modified) and a data-parallel style
    GRADS_ONLY step + apply_grads, each of which leaves the copies stale."""
    o1, e1 = make_hybrid_pair(algo, 64, 1000, 700, 71, graphs=False)
    o2, e2 = make_hybrid_pair(algo, 64, 1000, 700, 71, graphs=True)

    def both(fn):
        fn(e1)
        fn(e2)
    for i in range(7):
        both(lambda e: e.learn_step(soft_update=True))
        if i == 1:
            both(lambda e: e.hard_update())
        if i == 2:
            both(lambda e: e.soft_update())
        if i == 3:   # a host-side write through the torch views
            def poke(e):
                v = e.param_views(e.params)
                k = next(k for k in v if "cnn_stream.2.weight" in k)
                v[k].mul_(0.5)
                e.params_modified()
            both(poke)
        if i == 4:
            both(lambda e: e.learn_step(grads_only=True))
            both(lambda e: e.apply_grads(soft_update=True))
    torch.cuda.synchronize()
    e1.check_device_error()
    e2.check_device_error()
    assert torch.equal(e1.q, e2.q) and torch.equal(e1.grads, e2.grads)
    assert torch.equal(e1.params, e2.params) and torch.equal(e1.target_params, e2.target_params)


def _run_hybrid_steps(algo, batch, steps, seed):
    _, eng = make_hybrid_pair(algo, batch, 2000, 1500, seed)
    for _ in range(steps):
        eng.learn_step(soft_update=True)
    torch.cuda.synchronize()
    eng.check_device_error()
    out = [eng.params.cpu().clone(), eng.target_params.cpu().clone(), eng.q.cpu().clone()]
    del eng
    return out


@pytest.mark.parametrize("knob,a,b", [
    ("DQNX_MDX_WAVES", "8", "4"),    # micro data gradients: 8 vs 4 waves per workgroup
    ("DQNX_F1_ULOAD", "1", "0"),     # dense 1: unconditional float4 / float2-pair loads vs the guarded loader
    ("DQNX_F1_PF", "2", "1"),        # dense 1: two K passes in flight vs one
    ("DQNX_FWD_ULOAD", "1", "0"),    # dense 2: unconditional float4 loads vs the guarded loader
    ("DQNX_BWD_ULOAD", "1", "0"),    # dense backward: unconditional float4 / pair loads vs the guarded loader
    ("DQNX_BWD_TS", "64", "32"),     # dense-1 backward: 64 x 64 vs 32 x 32 tiles
    ("DQNX_MICRO_PIXPAD", "4", "8"), # micro forward / data gradients: LDS pixel stride Co + 4 vs Co + 8
])
@pytest.mark.parametrize("algo,batch", [("DuelingDoubleDQNAgent", 256), ("PerDuelingDoubleDQNAgent", 100)])
def test_gpu_hybrid_head_variants_bit_identical(monkeypatch, knob, a, b, algo, batch):
    """The HEAD net's launch variants change only where partial sums are combined or which wave
    computes an output, never the order of any sum: parameters, targets and Q-values stay bitwise
    equal over 4 steps."""
    monkeypatch.setenv(knob, a)
    ra = _run_hybrid_steps(algo, batch, 4, 41)
    monkeypatch.setenv(knob, b)
    rb = _run_hybrid_steps(algo, batch, 4, 41)
    for x, y, name in zip(ra, rb, ("params", "target", "q")):
        assert torch.equal(x, y), f"{knob}={a} vs {b}: {name} differ"
