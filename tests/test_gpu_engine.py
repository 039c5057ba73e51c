"""GPU parity: libdqnx (through its C ABI) against the oracle on seeded inputs."""
import ctypes
import os
import random

import numpy as np
import pytest
import torch

from oracle import ref as O
from parity import COMPARISONS, assert_grad_close, record_exemptions

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _engine_mod():
    from dqn import engine as E
    return E


def test_gpu_sampler_matches_oracle():
    from dqn import _capi as C
    L = C.lib()
    dev = torch.device("cuda")
    cases = [(50, 32), (200, 32), (4117, 1024), (4118, 1024), (10000, 1024), (100000, 4096),
             (1000000, 1024), (1000000, 8192), (16405, 4096), (16406, 4096), (7, 5), (6, 6), (1, 1),
             (3000, 0), (999, 999),
             # pipelined sampler (k <= 5984): acceptance ~1/2 (two rounds), its largest k, small k
             (524289, 4096), (524289, 5984), (1000000, 5984), (5000, 100), (2049, 600),
             # k beyond the LDS tables: the LDS-bitmap body (population <= 2^20; DQNX_SAMPLER_GLOBAL:
             # the global-memory hash table), incl. configs[3]'s weak-scaling draw (k = 32768 = 8 x 4096),
             # the bitmap's largest population and the pool branch at setsize(32768) = 262165
             (100000, 12000), (1000000, 16384), (1000000, 32768), (1048576, 32768), (300000, 32768),
             (262165, 32768), (1000000, 100000)]
    for j, (n, k) in enumerate(cases):
        random.seed(1000 + j)
        st = O.py_state_to_array()
        for rep in range(3):   # consecutive calls continue the same stream
            want_state = st.copy()
            want = O.sample_positions(want_state, n, k)
            d_state = torch.from_numpy(st.view(np.int32).copy()).to(dev)
            out = torch.zeros(max(k, 1), dtype=torch.int32, device=dev)
            err = torch.zeros(1, dtype=torch.int32, device=dev)
            scratch = torch.zeros(int(L.dqnx_sample_scratch_bytes(n, k)) + 16, dtype=torch.uint8, device=dev)
            C.check(L.dqnx_sample_uniform(d_state.data_ptr(), n, k, out.data_ptr(), scratch.data_ptr(),
                                          err.data_ptr(), torch.cuda.current_stream().cuda_stream), "sample")
            torch.cuda.synchronize()
            assert int(err.item()) == 0
            got = out.cpu().numpy()[:k].astype(np.int64)
            assert np.array_equal(got, want), (n, k, rep)
            new_state = d_state.cpu().numpy().view(np.uint32)
            assert np.array_equal(new_state, want_state), (n, k, rep)
            st = want_state


@pytest.mark.parametrize("mode", ["DQNX_SAMPLER_FORCE_FALLBACK", "DQNX_SAMPLER_OLD", "DQNX_SAMPLER_FAST",
                                  "DQNX_SAMPLER_GLOBAL"])
def test_gpu_sampler_other_paths_match_oracle(monkeypatch, mode):
    """The fast sampler's exact fallback (taken when a draw needs more words than the 8-sigma
    margin provides), the multi-pass kernel alone, and the fast path below its default k range,
    on the same cases."""
    monkeypatch.setenv(mode, "1")
    test_gpu_sampler_matches_oracle()


def test_gpu_sampler_golden():
    from dqn import _capi as C
    L = C.lib()
    z = np.load(os.path.join(GOLDEN, "sampler.npz"))
    for j in range(int(z["count"])):
        n, k = int(z[f"c{j}_n"]), int(z[f"c{j}_k"])
        d_state = torch.from_numpy(z[f"c{j}_state_in"].view(np.int32).copy()).cuda()
        out = torch.zeros(k, dtype=torch.int32, device="cuda")
        err = torch.zeros(1, dtype=torch.int32, device="cuda")
        scratch = torch.zeros(int(L.dqnx_sample_scratch_bytes(n, k)) + 16, dtype=torch.uint8, device="cuda")
        C.check(L.dqnx_sample_uniform(d_state.data_ptr(), n, k, out.data_ptr(), scratch.data_ptr(),
                                      err.data_ptr(), torch.cuda.current_stream().cuda_stream), "sample")
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().astype(np.int64), z[f"c{j}_idx"]), j
        assert np.array_equal(d_state.cpu().numpy().view(np.uint32), z[f"c{j}_state_out"]), j


def test_gpu_sampler_k_larger_than_n_sets_error():
    from dqn import _capi as C
    L = C.lib()
    d_state = torch.from_numpy(O.py_state_to_array().view(np.int32).copy()).cuda()
    before = d_state.clone()
    out = torch.zeros(8, dtype=torch.int32, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    scratch = torch.zeros(int(L.dqnx_sample_scratch_bytes(5, 8)) + 16, dtype=torch.uint8, device="cuda")
    C.check(L.dqnx_sample_uniform(d_state.data_ptr(), 5, 8, out.data_ptr(), scratch.data_ptr(), err.data_ptr(),
                                  torch.cuda.current_stream().cuda_stream), "sample")
    torch.cuda.synchronize()
    assert int(err.item()) == C.DEVERR_SAMPLE_TOO_LARGE
    assert torch.equal(before, d_state)   # ValueError consumes nothing


def make_pair(algo, obs_dim, batch, capacity, n_fill, seed, graphs=True):
    E = _engine_mod()
    head = O.algo_spec_head(algo)
    ospec = O.mlp_spec(obs_dim, 8, head)
    init = O.reference_init(ospec, seed)
    oracle = O.OracleLearner(ospec, algo, batch, capacity, seed=seed, params=init)
    data = O.synth_transitions(n_fill, obs_dim, 8, seed=seed + 100)
    O.fill_replay(oracle, *data)
    eng = E.LearnEngine(E.mlp_spec(obs_dim, 8, head), algo, batch, capacity, graphs=graphs)
    eng.load_params(init)
    obs, act, rew, done, new_obs = data
    eng.push(obs, act, rew, done, new_obs)
    random.seed(seed + 7)
    st = O.py_state_to_array()
    oracle.py_state = st.copy()
    eng.set_rng(0, st)
    return oracle, eng


LOOSE_MAX_FRAC = 1e-3   # at most 0.1 % of a tensor's entries may use the 2 lr bound


def compare_state(oracle, eng, atol=1e-5, loose=None, report=None):
    """Weights within atol, Adam m / v within 1e-6 / 1e-7.  `loose` (from _check_learn): per
    tensor, the entries whose gradient differed by more than 0.1 % in some step.  Adam moves a
    weight by about lr * g / |g| whatever the size of g, so there the step is not determined to
    1e-5 by a gradient that agrees to the gradient tolerance (a ReLU mask flipped by an fp32
    pre-activation within rounding of zero does this); those entries are bounded by 2 lr per
    step instead, everything else by atol.  Only the exempted entries that actually exceed atol
    are counted; more than LOOSE_MAX_FRAC of a tensor fails the test, and the counts are
    returned (and printed) so the exemption is never silent."""
    views = {"online": eng.param_views(eng.params), "target": eng.param_views(eng.target_params),
             "m": eng.param_views(eng.adam_m), "v": eng.param_views(eng.adam_v)}
    COMPARISONS[0] += 1
    worst = {}
    exempt = {}
    for nm, src in (("online", oracle.online), ("target", oracle.target), ("m", oracle.m), ("v", oracle.v)):
        for k, ref in src.items():
            got = views[nm][k].detach().cpu()
            d = (got - ref).abs()
            if nm in ("online", "target") and loose is not None and bool(loose[k].any()):
                over = loose[k] & (d > atol)
                n_over = int(over.sum())
                if n_over:
                    assert float(d[over].max()) <= 2.0 * oracle.lr + atol, (nm, k)   # one step from synced state
                    exempt[f"{nm}:{k}"] = n_over
                    assert n_over <= LOOSE_MAX_FRAC * d.numel(), (nm, k, n_over, d.numel())
                d = d * (~loose[k])
            worst[nm] = max(worst.get(nm, 0.0), float(d.max()))
    if exempt:
        print("exempted entries (2 lr bound):", exempt)
        numels = {f"{nm}:{k}": views[nm][k].numel() for nm in ("online", "target") for k in oracle.online}
        record_exemptions(exempt, numels)
    if report is not None:
        report.update(exempt)
    assert worst["online"] <= atol and worst["target"] <= atol, worst
    assert worst["m"] <= 1e-6 and worst["v"] <= 1e-7, worst
    return worst


@pytest.mark.parametrize("algo,obs_dim,batch,capacity,n_fill,seed", [
    ("DQNAgent", 14, 32, 500, 300, 3),
    ("DoubleDQNAgent", 14, 32, 500, 300, 4),
    ("DuelingDoubleDQNAgent", 14, 32, 500, 300, 5),
    ("DuelingDoubleDQNAgent", 284, 256, 5000, 3000, 6),
    ("DuelingDoubleDQNAgent", 284, 1024, 20000, 20000, 7),
    ("DoubleDQNAgent", 284, 100, 700, 650, 8),
    ("DuelingDoubleDQNAgent", 284, 4096, 60000, 60000, 19),   # configs[3]'s global minibatch
])
def test_gpu_learn_matches_oracle(algo, obs_dim, batch, capacity, n_fill, seed):
    _check_learn(*make_pair(algo, obs_dim, batch, capacity, n_fill, seed))


@pytest.mark.parametrize("algo,obs_dim,batch,capacity,n_fill,seed", [
    ("DQNAgent", 14, 32, 500, 300, 13),
    ("DuelingDoubleDQNAgent", 284, 1024, 20000, 20000, 17),
])
def test_gpu_learn_fused_backward_plan_matches_oracle(monkeypatch, algo, obs_dim, batch, capacity, n_fill, seed):
    """Backward plan 1 (head kernel makes dZ_{L-1}; one full-K dW + Adam launch)."""
    monkeypatch.setenv("DQNX_BWD_PLAN", "1")
    _check_learn(*make_pair(algo, obs_dim, batch, capacity, n_fill, seed))


@pytest.mark.parametrize("dw16,algo,obs_dim,batch,capacity,n_fill,seed", [
    ("0", "DuelingDoubleDQNAgent", 284, 256, 3000, 3000, 61),    # split-K slabs + Adam pass
    ("0", "DQNAgent", 14, 100, 500, 300, 62),
    ("1", "DuelingDoubleDQNAgent", 284, 4096, 60000, 60000, 63),   # full-K tiles past 2048 rows
    ("1", "DoubleDQNAgent", 284, 1000, 20000, 20000, 64),          # ragged K tail
])
def test_gpu_learn_dw_plans_match_oracle(monkeypatch, dw16, algo, obs_dim, batch, capacity, n_fill, seed):
    """Both weight-gradient routes of the fused plan: k_dw_adam16 (full-minibatch 16 x 16 tiles,
    Adam and the blocked copies in one launch; default up to 2048 rows) and the split-K slabs +
    Adam pass (default beyond), each forced at a batch where the other is the default."""
    monkeypatch.setenv("DQNX_DW_ADAM16", dw16)
    _check_learn(*make_pair(algo, obs_dim, batch, capacity, n_fill, seed))


@pytest.mark.parametrize("algo,obs_dim,batch,capacity,n_fill,seed", [
    ("DQNAgent", 14, 32, 500, 300, 23),
    ("DoubleDQNAgent", 284, 256, 3000, 3000, 24),
    ("DuelingDoubleDQNAgent", 284, 1000, 20000, 20000, 25),   # ragged last tile
])
def test_gpu_learn_per_layer_plan_matches_oracle(monkeypatch, algo, obs_dim, batch, capacity, n_fill, seed):
    """Plan 0 (per-layer forward launches + split-K backward levels), the plan two-stream nets use."""
    monkeypatch.setenv("DQNX_BWD_PLAN", "0")
    _check_learn(*make_pair(algo, obs_dim, batch, capacity, n_fill, seed))


@pytest.mark.parametrize("mr", ["1", "2", "4"])
@pytest.mark.parametrize("algo,obs_dim,batch,capacity,n_fill,seed", [
    ("DuelingDoubleDQNAgent", 284, 1000, 20000, 20000, 41),   # ragged last row tile
    ("DQNAgent", 14, 100, 500, 300, 42),
])
def test_gpu_learn_forward_row_tiles_match_oracle(monkeypatch, mr, algo, obs_dim, batch, capacity, n_fill, seed):
    """Fused forward with 16- / 32- / 64-row workgroups (one launch: no layer-1 split)."""
    monkeypatch.setenv("DQNX_FWD_MR", mr)
    monkeypatch.setenv("DQNX_FWD_SPLIT", "1")
    _check_learn(*make_pair(algo, obs_dim, batch, capacity, n_fill, seed))


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
@pytest.mark.parametrize("split", ["2", "4"])
def test_gpu_split_forward_identical(monkeypatch, split, compute):
    """Layer 1 in a launch of its own over 2 / 4 column parts (H_1 through HBM) gives bitwise
    the same steps as the one-launch forward; ragged batch."""
    E = _engine_mod()
    outs = []
    for sp in (split, "1"):
        monkeypatch.setenv("DQNX_FWD_SPLIT", sp)
        o, e = make_pair("DuelingDoubleDQNAgent", 284, 1000, 20000, 20000, 44)
        if compute == "bf16":
            e = E.LearnEngine(E.mlp_spec(284, 8, "dueling"), "DuelingDoubleDQNAgent", 1000, 20000,
                              compute_dtype="bf16")
            e.load_params(O.reference_init(O.mlp_spec(284, 8, "dueling"), 44))
            e.push(*O.synth_transitions(20000, 284, 8, seed=144))
            random.seed(51)
            e.set_rng(0, O.py_state_to_array())
        for _ in range(3):
            e.learn_step(soft_update=True)
        torch.cuda.synchronize()
        outs.append((e.params.clone(), e.q.clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("algo,batch", [("DuelingDoubleDQNAgent", 1024), ("DuelingDoubleDQNAgent", 1020),
                                        ("DQNAgent", 1024), ("DoubleDQNAgent", 4096)])
def test_gpu_pair_forward_identical(monkeypatch, algo, batch):
    """DQNX_FWD_PAIR=1: the one-launch forward with layer 1's columns over two partner workgroups
    and the in-launch hand-off of the H_1 halves gives bitwise the same steps as the default
    forward, over enough steps that every hand-off word is reused; ragged last tile at 1020."""
    outs = []
    for pair in ("1", "0"):
        monkeypatch.setenv("DQNX_FWD_PAIR", pair)
        o, e = make_pair(algo, 284, batch, 20000, 20000, 45)
        for _ in range(8):
            e.learn_step(soft_update=True)
        torch.cuda.synchronize()
        e.check_device_error()
        outs.append((e.params.clone(), e.target_params.clone(), e.q.clone()))
    for x, y in zip(outs[0], outs[1]):
        assert torch.equal(x, y)


@pytest.mark.parametrize("split", ["2", "4"])
def test_gpu_fused_head_split_identical(monkeypatch, split):
    """The fused plan's head/dZ-chain kernel with the last dZ split over 2 or 4 workgroups per
    tile gives bitwise the same step as unsplit (each column is computed the same way)."""
    monkeypatch.setenv("DQNX_HEAD_SPLIT", split)
    o, e = make_pair("DuelingDoubleDQNAgent", 284, 512, 4000, 4000, 31)
    monkeypatch.setenv("DQNX_HEAD_SPLIT", "1")
    o2, e2 = make_pair("DuelingDoubleDQNAgent", 284, 512, 4000, 4000, 31)
    for _ in range(3):
        e.learn_step(soft_update=True)
        e2.learn_step(soft_update=True)
    torch.cuda.synchronize()
    assert torch.equal(e.params, e2.params)
    assert torch.equal(e.target_params, e2.target_params)


def sync_oracle(oracle, eng):
    """Continue the oracle from the engine's state, so every step is checked from identical
    inputs.  Without it, one legitimate 2*lr difference (see compare_state) feeds the next
    forward and the trajectories drift apart by more than one step's tolerance."""
    views = {"online": eng.param_views(eng.params), "target": eng.param_views(eng.target_params),
             "m": eng.param_views(eng.adam_m), "v": eng.param_views(eng.adam_v)}
    for nm, dst in (("online", oracle.online), ("target", oracle.target), ("m", oracle.m), ("v", oracle.v)):
        for k in dst:
            dst[k].copy_(views[nm][k].detach().cpu())


def _check_learn(oracle, eng):
    loose = {}
    for step in range(3):
        rec = oracle.train_step()
        eng.learn_step(soft_update=True)
        torch.cuda.synchronize()
        eng.check_device_error()
        idx = eng.batch_idx.cpu().numpy().astype(np.int64)
        assert np.array_equal(idx, rec.positions), f"step {step}: sampled indices differ"
        q = eng.q.cpu()
        np.testing.assert_allclose(q[0].numpy(), rec.q_online.numpy(), atol=1e-5, rtol=0)
        np.testing.assert_allclose(q[2].numpy(), rec.q_target_next.numpy(), atol=1e-5, rtol=0)
        if rec.q_online_next is not None:
            np.testing.assert_allclose(q[1].numpy(), rec.q_online_next.numpy(), atol=1e-5, rtol=0)
        np.testing.assert_allclose(eng.td[0].cpu().numpy(), rec.targets.view(-1).numpy(), atol=1e-5, rtol=0)
        assert abs(eng.loss() - rec.loss) <= 1e-5 * max(1.0, abs(rec.loss))
        g = eng.param_views(eng.grads[:-1])
        for k, ref in rec.grads.items():
            gk = g[k].cpu()
            assert_grad_close(gk.numpy(), ref.numpy(), f"{k} step {step}")
            loose[k] = (gk - ref).abs() > 1e-3 * ref.abs() + 1e-9
        compare_state(oracle, eng, loose=loose)
        sync_oracle(oracle, eng)
    assert np.array_equal(eng.get_rng(0), oracle.py_state)


@pytest.mark.parametrize("adam_blk,dw16", [("0", "1"), ("0", "0"), ("1", "0")])
@pytest.mark.parametrize("compute", ["fp32", "bf16"])
def test_gpu_weights_written_from_host_are_used(monkeypatch, compute, adam_blk, dw16):
    """The fused plan keeps fragment-blocked weight copies current from the Adam pass; weights
    written from the host (a checkpoint load through load_params / state_dict views, hard or
    soft updates) must reach the next step's forward (DQNX_STEP relayout after
    dqnx_params_modified).  Checked by loading fresh weights mid-run into engine and oracle,
    with the copies maintained by k_dw_adam16 (default), rebuilt every step (slab plan) and
    maintained by the slab plan's Adam pass (DQNX_ADAM_BLK=1)."""
    monkeypatch.setenv("DQNX_ADAM_BLK", adam_blk)
    monkeypatch.setenv("DQNX_DW_ADAM16", dw16)
    o, e = make_pair("DuelingDoubleDQNAgent", 284, 256, 3000, 3000, 27)
    if compute == "bf16":   # bf16: only that the host-written weights are the ones used
        E = _engine_mod()
        e = E.LearnEngine(E.mlp_spec(284, 8, "dueling"), "DuelingDoubleDQNAgent", 256, 3000, compute_dtype="bf16")
        e.push(*O.synth_transitions(3000, 284, 8, seed=127))
        random.seed(3)
        e.set_rng(0, O.py_state_to_array())
    e.load_params(O.reference_init(O.mlp_spec(284, 8, "dueling"), 27))
    e.learn_step(soft_update=True)
    if compute == "fp32":
        o.train_step()
    fresh = O.reference_init(O.mlp_spec(284, 8, "dueling"), 99)
    e.load_params(fresh)
    if compute == "bf16":
        # the first forward after the load equals a forward of a fresh engine holding `fresh`
        e2 = _engine_mod().LearnEngine(e.spec, "DuelingDoubleDQNAgent", 256, 3000, compute_dtype="bf16")
        e2.push(*O.synth_transitions(3000, 284, 8, seed=127))
        e2.load_params(fresh)
        e2.set_rng(0, e.get_rng(0))
        e.learn_step(soft_update=True)
        e2.learn_step(soft_update=True)
        torch.cuda.synchronize()
        assert torch.equal(e.q, e2.q)
        return
    for k in o.online:
        o.online[k].copy_(fresh[k])
        o.target[k].copy_(fresh[k])
    rec = o.train_step()
    e.learn_step(soft_update=True)
    torch.cuda.synchronize()
    np.testing.assert_allclose(e.q[0].cpu().numpy(), rec.q_online.numpy(), atol=1e-5, rtol=0)
    np.testing.assert_allclose(e.q[2].cpu().numpy(), rec.q_target_next.numpy(), atol=1e-5, rtol=0)
    # a hard update (target <- online) is seen by the next step's target forward too
    e.hard_update()
    for k in o.online:
        o.target[k].copy_(o.online[k])
    sync_oracle(o, e)
    rec = o.train_step()
    e.learn_step(soft_update=True)
    torch.cuda.synchronize()
    np.testing.assert_allclose(e.q[2].cpu().numpy(), rec.q_target_next.numpy(), atol=1e-5, rtol=0)


def test_gpu_learn_graph_and_eager_identical():
    o1, e1 = make_pair("DuelingDoubleDQNAgent", 284, 512, 4000, 4000, 11, graphs=True)
    o2, e2 = make_pair("DuelingDoubleDQNAgent", 284, 512, 4000, 4000, 11, graphs=False)
    for _ in range(4):
        e1.learn_step(soft_update=True)
        e2.learn_step(soft_update=True)
    torch.cuda.synchronize()
    assert torch.equal(e1.params, e2.params)
    assert torch.equal(e1.target_params, e2.target_params)


GOLDEN_MLP = ["learn_mlp14_DQNAgent", "learn_mlp14_DoubleDQNAgent", "learn_mlp14_DuelingDoubleDQNAgent",
              "learn_mlp284_DuelingDoubleDQNAgent", "learn_mlp284b1024_DuelingDoubleDQNAgent",
              "learn_mlp284b4096_DuelingDoubleDQNAgent", "learn_mlp284b8192_PerDuelingDoubleDQNAgent"]


@pytest.mark.parametrize("golden", GOLDEN_MLP)
def test_gpu_learn_golden(golden):
    """Engine against the reference's own outputs (tests/golden, made by make_golden.py by
    running the reference): sampled positions / tree leaves and RNG state bit-exact, loss and
    the online and target weights after every step within a strict 1e-5 (no exemptions).
    Covers configs[1]'s batch (1024), configs[3]'s global batch (4096) and configs[4]'s PER
    batch (8192, fp32 arithmetic)."""
    E = _engine_mod()
    z = np.load(os.path.join(GOLDEN, golden + ".npz"))
    algo = str(z["algo"])
    per = algo.startswith("Per")
    obs_dim, batch, cap = int(z["obs_dim"]), int(z["batch"]), int(z["buffer"])
    head = O.algo_spec_head(algo)
    init = O.reference_init(O.mlp_spec(obs_dim, 8, head), int(z["seed"]))
    eng = E.LearnEngine(E.mlp_spec(obs_dim, 8, head), algo, batch, cap)
    eng.load_params(init)
    eng.push(*O.synth_transitions(int(z["n_fill"]), obs_dim, 8, seed=int(z["seed"]) + 100))
    eng.set_rng(0, z["py_state_in"])
    eng.set_rng(1, z["np_state_in"])
    for s in range(int(z["steps"])):
        eng.learn_step(soft_update=True)
        torch.cuda.synchronize()
        eng.check_device_error()
        got = eng.batch_idx.cpu().numpy().astype(np.int64) + (cap - 1 if per else 0)
        assert np.array_equal(got, z["pos"][s]), f"step {s}: positions differ"
        if per:
            # step 1 samples a tree of pushed max priorities: exact to fp32 rounding.  Later steps
            # weight by (p / p_min)^-beta, and p_min = (|delta_min| + 1e-4)^0.6 comes from a small
            # |delta| that carries the forward's fp32 noise amplified by dp/d|delta| (<= 24)
            rtol = 1e-6 if s == 0 else 1e-5
            np.testing.assert_allclose(eng.is_weights.cpu().numpy(), z["isw"][s].astype(np.float32), rtol=rtol)
        assert abs(eng.loss() - z["loss"][s]) <= 1e-5 * max(1.0, abs(z["loss"][s])), (s, eng.loss(), z["loss"][s])
    if per:
        assert np.array_equal(eng.get_rng(1), z["np_state_out"])
    else:
        assert np.array_equal(eng.get_rng(0), z["py_state_out"])
    stride = int(z["stride"])
    keys = [str(k) for k in z["keys"]]
    on, tg = eng.param_views(eng.params), eng.param_views(eng.target_params)
    for i, k in enumerate(keys):
        for nm, views in (("online", on), ("target", tg)):
            got = views[k].cpu().numpy().reshape(-1)
            ref = z[f"{nm}_{i}"]
            if got.size != ref.size:
                got = got[::stride]
            np.testing.assert_allclose(got, ref, atol=1e-5, rtol=0, err_msg=f"{nm} {k}")


@pytest.mark.parametrize("plan,batch,graphs", [("0", 256, True), ("fused", 256, True), ("fused", 1024, True),
                                               ("fused", 1024, False), ("fused", 2048, True), ("fused", 4096, False)])
def test_gpu_prefetch_mode_bit_identical(monkeypatch, plan, batch, graphs):
    """DQNX_STEP_PREFETCH draws step t+1's minibatch during step t: same results, bitwise.
    Per-layer plan: a side-stream pipeline.  Fused plan: step t's k_dw_adam16 launch hosts step
    t+1's sampler workgroup (in-launch prefetch; B=2048 is its largest k)."""
    if plan == "0":
        monkeypatch.setenv("DQNX_BWD_PLAN", "0")
    n = max(3000, 2 * batch)
    o1, e1 = make_pair("DuelingDoubleDQNAgent", 284, batch, n, n, 21)
    o2, e2 = make_pair("DuelingDoubleDQNAgent", 284, batch, n, n, 21, graphs=graphs)
    for _ in range(6):
        e1.learn_step(soft_update=True)
    for _ in range(5):
        e2.learn_step(soft_update=True, prefetch=True)
    e2.learn_step(soft_update=True)     # consumes the pending minibatch
    torch.cuda.synchronize()
    e1.check_device_error()
    e2.check_device_error()
    assert torch.equal(e1.params, e2.params)
    assert torch.equal(e1.target_params, e2.target_params)
    assert np.array_equal(e1.get_rng(0), e2.get_rng(0))
    # after the flush, pushes are allowed again
    e2.push(*O.synth_transitions(4, 284, 8, seed=3))


@pytest.mark.parametrize("algo,batch,count,n_fill", [
    ("DuelingDoubleDQNAgent", 4096, 3, 9000),     # slab plan: Adam pass copies, relayout launches
    ("DuelingDoubleDQNAgent", 1024, 1, 4000),
    ("DuelingDoubleDQNAgent", 1024, 2, 4000),
    ("DuelingDoubleDQNAgent", 1024, 7, 4000),
    ("DQNAgent", 256, 4, 3000),
    ("DuelingDoubleDQNAgent", 1024, 3, 3000),     # n <= setsize: the pool branch in-launch
    ("PerDuelingDoubleDQNAgent", 256, 3, 3000),   # no in-launch sampler: steps one by one
])
def test_gpu_learn_steps_equal_single_steps(algo, batch, count, n_fill):
    """dqnx_learn_steps(count) == count x dqnx_learn_step, bitwise (weights, target, Adam state,
    loss, RNG), with host-side weight writes before the call (relayout in the graph's sampler)."""
    o1, e1 = make_pair(algo, 284, batch, max(n_fill, 3000), n_fill, 31)
    o2, e2 = make_pair(algo, 284, batch, max(n_fill, 3000), n_fill, 31)
    for rnd in range(2):
        for _ in range(count):
            e1.learn_step(soft_update=True)
        e2.learn_steps(count, soft_update=True)
        torch.cuda.synchronize()
        e1.check_device_error()
        e2.check_device_error()
        assert torch.equal(e1.params, e2.params), rnd
        assert torch.equal(e1.target_params, e2.target_params), rnd
        assert torch.equal(e1.adam_m, e2.adam_m) and torch.equal(e1.adam_v, e2.adam_v), rnd
        assert e1.loss() == e2.loss()
        assert np.array_equal(e1.get_rng(0), e2.get_rng(0))
        if algo.startswith("Per"):
            assert np.array_equal(e1.get_rng(1), e2.get_rng(1))
        new = O.reference_init(O.mlp_spec(284, 8, O.algo_spec_head(algo)), 50 + rnd)
        e1.load_params(new)
        e2.load_params(new)
    # nothing is pending afterwards: pushes are allowed
    e2.push(*O.synth_transitions(4, 284, 8, seed=3))


@pytest.mark.parametrize("world,k", [(8, 4096), (4, 4096), (2, 4096), (2, 2048), (1, 4096)])
def test_gpu_prefetch_dp_shard_step_bit_identical(world, k):
    """configs[3] shard step (rank 0 of `world`, global minibatch k): the next GLOBAL minibatch
    drawn inside the forward launch (k = 4096: one-pass 16384-slot table while the grid leaves a CU
    idle, 8192-slot passes at 2048 rows per rank; k = 2048: 4096 slots) gives the same
    gradients and weights as the sampler launch, bitwise."""
    E = _engine_mod()
    ospec = O.mlp_spec(284, 8, "dueling")
    init = O.reference_init(ospec, 41)
    data = O.synth_transitions(12000, 284, 8, seed=141)
    engines = []
    for _ in range(2):
        eng = E.LearnEngine(E.mlp_spec(284, 8, "dueling"), "DuelingDoubleDQNAgent", k, 12000,
                            world_size=world, rank=0)
        eng.load_params(init)
        eng.push(*data)
        random.seed(48)
        eng.set_rng(0, O.py_state_to_array())
        engines.append(eng)
    e1, e2 = engines
    for i in range(4):
        e1.learn_step(grads_only=True)
        e1.apply_grads(soft_update=True)
        e2.learn_step(grads_only=True, prefetch=i < 3)
        e2.apply_grads(soft_update=True)
    torch.cuda.synchronize()
    e1.check_device_error()
    e2.check_device_error()
    assert torch.equal(e1.grads, e2.grads)
    assert torch.equal(e1.params, e2.params) and torch.equal(e1.target_params, e2.target_params)
    assert np.array_equal(e1.get_rng(0), e2.get_rng(0))


@pytest.mark.parametrize("world,n,cap,rolled", [(8, 260000, None, "0"), (4, 260000, None, "0"),
                                                (8, 150000, None, "0"), (8, 260000, "2", "0"),
                                                (8, 260000, "-1", "0"), (8, 260000, None, "1"),
                                                (4, 150000, None, "1"), (8, 260000, "2", "1")])
def test_gpu_prefetch_bitmap_first_pass_bit_identical(monkeypatch, world, n, cap, rolled):
    """The in-forward draw's bitmap first pass (one-pass shape, n <= 2^20 and n >= 32 k): exact
    "seen" bits plus the repeat table give the same positions and RNG state as the sampler launch,
    bitwise.  n = 260000: one pass; n = 150000: 1.75 words per draw, so the draw continues on the
    hash table seeded from the first pass; DQNX_SAMPLER_BM_CAP=2: more repeats than the cap, the
    pass redone on the hash table; -1: the bitmap pass off.  DQNX_SAMPLER_ROLLED: either form of the
    bitmap pass (unrolled register arrays / rolled loops over bit masks)."""
    monkeypatch.setenv("DQNX_SAMPLER_ROLLED", rolled)
    if cap is not None:
        monkeypatch.setenv("DQNX_SAMPLER_BM_CAP", cap)
    E = _engine_mod()
    k = 4096
    ospec = O.mlp_spec(32, 8, "dueling")
    init = O.reference_init(ospec, 43)
    data = O.synth_transitions(n, 32, 8, seed=143)
    engines = []
    for _ in range(2):
        eng = E.LearnEngine(E.mlp_spec(32, 8, "dueling"), "DuelingDoubleDQNAgent", k, n,
                            world_size=world, rank=0)
        eng.load_params(init)
        eng.push(*data)
        random.seed(49)
        eng.set_rng(0, O.py_state_to_array())
        engines.append(eng)
    e1, e2 = engines
    for i in range(4):
        e1.learn_step(grads_only=True)
        e1.apply_grads(soft_update=True)
        e2.learn_step(grads_only=True, prefetch=i < 3)
        e2.apply_grads(soft_update=True)
    torch.cuda.synchronize()
    e1.check_device_error()
    e2.check_device_error()
    assert torch.equal(e1.grads, e2.grads)
    assert torch.equal(e1.params, e2.params) and torch.equal(e1.target_params, e2.target_params)
    assert np.array_equal(e1.get_rng(0), e2.get_rng(0))


@pytest.mark.parametrize("algo,batch", [("DuelingDoubleDQNAgent", 1024), ("DQNAgent", 200),
                                        ("PerDuelingDoubleDQNAgent", 512)])
def test_gpu_dw16_row_pair_tiles_bit_identical(monkeypatch, algo, batch):
    """k_dw_adam16 on 32 x 16 tiles (the default: two 16-row blocks of W share each X load) sums
    every gradient in the same order as the 16 x 16 tiles (DQNX_DW16_R=1): weights, target, Adam
    state and gradients are bitwise equal."""
    monkeypatch.setenv("DQNX_DW16_R", "1")
    o1, e1 = make_pair(algo, 284, batch, 3000, 3000, 81)
    for _ in range(3):
        e1.learn_step(soft_update=True)   # (the plan is built at the first step)
    torch.cuda.synchronize()
    monkeypatch.delenv("DQNX_DW16_R")
    o2, e2 = make_pair(algo, 284, batch, 3000, 3000, 81)
    for _ in range(3):
        e2.learn_step(soft_update=True)
    torch.cuda.synchronize()
    e1.check_device_error()
    e2.check_device_error()
    assert torch.equal(e1.grads, e2.grads)
    assert torch.equal(e1.params, e2.params) and torch.equal(e1.target_params, e2.target_params)
    assert torch.equal(e1.adam_m, e2.adam_m) and torch.equal(e1.adam_v, e2.adam_v)


@pytest.mark.parametrize("algo,batch,prefetch", [("DuelingDoubleDQNAgent", 1024, True),
                                                 ("DuelingDoubleDQNAgent", 512, False),
                                                 ("PerDuelingDoubleDQNAgent", 1024, False)])
def test_gpu_xcd_row_mapping_bit_identical(monkeypatch, algo, batch, prefetch):
    """The XCD-aligned row tiles (default: row tile t of every stream and the head's tile t on XCD
    t % 8) only move workgroups: results are bitwise those of xcd_remap's order (DQNX_XCD_ROWS=0)."""
    monkeypatch.setenv("DQNX_XCD_ROWS", "0")
    o1, e1 = make_pair(algo, 284, batch, 3000, 3000, 83)
    for i in range(3):
        e1.learn_step(soft_update=True, prefetch=prefetch and i < 2)
    torch.cuda.synchronize()
    monkeypatch.delenv("DQNX_XCD_ROWS")
    o2, e2 = make_pair(algo, 284, batch, 3000, 3000, 83)
    for i in range(3):
        e2.learn_step(soft_update=True, prefetch=prefetch and i < 2)
    torch.cuda.synchronize()
    e1.check_device_error()
    e2.check_device_error()
    assert torch.equal(e1.q, e2.q) and torch.equal(e1.td, e2.td)
    assert torch.equal(e1.params, e2.params) and torch.equal(e1.target_params, e2.target_params)


def test_gpu_prefetch_fused_weights_written_while_pending():
    """Fused plan, in-launch prefetch: host-side weight writes (load_params) while a minibatch is
    pending rebuild the blocked copies before the next step, and the step matches a sequential
    engine that got the same write."""
    o1, e1 = make_pair("DuelingDoubleDQNAgent", 284, 1024, 4000, 4000, 23)
    o2, e2 = make_pair("DuelingDoubleDQNAgent", 284, 1024, 4000, 4000, 23)
    e1.learn_step(soft_update=True)
    e2.learn_step(soft_update=True, prefetch=True)
    new = O.reference_init(O.mlp_spec(284, 8, "dueling"), 99)
    e1.load_params(new)
    e2.load_params(new)
    for _ in range(2):
        e1.learn_step(soft_update=True)
    e2.learn_step(soft_update=True, prefetch=True)
    e2.learn_step(soft_update=True)
    torch.cuda.synchronize()
    assert torch.equal(e1.params, e2.params)
    assert torch.equal(e1.target_params, e2.target_params)
    assert abs(e1.loss() - e2.loss()) == 0.0


@pytest.mark.parametrize("plan", ["0", "fused"])
def test_gpu_push_refused_with_pending_prefetch(monkeypatch, plan):
    from dqn import _capi as C
    if plan == "0":
        monkeypatch.setenv("DQNX_BWD_PLAN", "0")
    o, e = make_pair("DuelingDoubleDQNAgent", 14, 32, 500, 300, 22)
    e.learn_step(prefetch=True)
    with pytest.raises(C.DqnxError):
        e.push(*O.synth_transitions(2, 14, 8, seed=1))
    e.learn_step()
    torch.cuda.synchronize()


@pytest.mark.parametrize("world,k", [(8, 4096), (1, 1024), (2, 1024)])
def test_gpu_apply_grads_tiles_bit_identical(monkeypatch, world, k):
    """dqnx_apply_grads on the fused plan with a prefetched minibatch pending (the DP shard step):
    k_dw_adam16 in apply mode (32 x 16 tiles, blocked copies per tile, the default) against k_adam's
    per-element pass (DQNX_APPLY_TILES=0): the same update and blocked copies, so every later step
    is bitwise equal too."""
    E = _engine_mod()
    ospec = O.mlp_spec(284, 8, "dueling")
    init = O.reference_init(ospec, 43)
    data = O.synth_transitions(9000, 284, 8, seed=143)
    engines = []
    for tiles in ("0", "1"):
        monkeypatch.setenv("DQNX_APPLY_TILES", tiles)
        eng = E.LearnEngine(E.mlp_spec(284, 8, "dueling"), "DuelingDoubleDQNAgent", k, 9000,
                            world_size=world, rank=0)
        eng.load_params(init)
        eng.push(*data)
        random.seed(49)
        eng.set_rng(0, O.py_state_to_array())
        for i in range(4):
            eng.learn_step(grads_only=True, prefetch=i < 3)
            eng.apply_grads(soft_update=True)
        torch.cuda.synchronize()
        eng.check_device_error()
        engines.append(eng)
    e1, e2 = engines
    assert torch.equal(e1.q, e2.q) and torch.equal(e1.grads, e2.grads)
    assert torch.equal(e1.params, e2.params) and torch.equal(e1.target_params, e2.target_params)
    assert torch.equal(e1.adam_m, e2.adam_m) and torch.equal(e1.adam_v, e2.adam_v)
    assert e1.loss() == e2.loss()



@pytest.mark.parametrize("batch,world,cap,graph_steps,knobs", [
    (8192, 1, 30000, 0, "DQNX_PF_SIDE_MIN_K=0"), (32768, 8, 300000, 0, ""), (32768, 8, 300000, 3, ""),
    # the side pipeline's alternative routes: fork / draw-done as marker packets (+ the compute
    # launches eager), and the apply leaving the blocked copies to a relayout launch
    (32768, 8, 300000, 0, "DQNX_SIDE_EXTEV=0"), (32768, 8, 300000, 0, "DQNX_SIDE_EXTEV=0,DQNX_SIDE_GRAPH=0"),
    (32768, 8, 300000, 0, "DQNX_SIDE_APPLY_KEEP=0"), (8192, 1, 30000, 0, "DQNX_SIDE_APPLY_KEEP=0,DQNX_PF_SIDE_MIN_K=0"),
    (16384, 4, 300000, 0, ""), (8192, 2, 300000, 0, "")])   # (k = 8192: the draw as its own launch)
def test_gpu_side_prefetch_bit_identical(batch, world, cap, graph_steps, knobs, monkeypatch):
    """The fused plan's side-stream prefetch (k beyond the forward's sampler workgroup: step t+1's
    random.sample drawn on the engine's side stream beside step t, then copied over the compute slot):
    bitwise the same weights, target, RNG state and minibatch as sequential steps -- one GPU at B = 8192,
    and rank 0 of world 8 at configs[3]'s weak-scaling global 32768 (the LDS-bitmap sampler), eager and
    as a captured graph of an odd number of steps.  R:dqn/replay_memory.py:38-39, R:dqn/agent.py:204-226."""
    from dqn import data_parallel as DP
    for kv in filter(None, knobs.split(",")):
        monkeypatch.setenv(*kv.split("="))
    E = _engine_mod()
    spec = E.mlp_spec(284, 8, "dueling")
    data = O.synth_transitions(cap, 284, 8, seed=3)
    init = O.reference_init(O.mlp_spec(284, 8, "dueling"), 4)

    def make():
        e = E.LearnEngine(spec, "DuelingDoubleDQNAgent", batch, cap, world_size=world, rank=0)
        e.load_params(init)
        e.push(*data)
        random.seed(77)
        e.set_rng(0, np.array(random.getstate()[1], dtype=np.uint32))
        return e

    def step(e, pf):
        if world > 1:
            e.learn_step(grads_only=True, prefetch=pf)
            e.apply_grads(soft_update=True)
        else:
            e.learn_step(soft_update=True, prefetch=pf)

    a = make()
    for _ in range(7):
        step(a, False)
    torch.cuda.synchronize()
    a.check_device_error()
    b = make()
    if graph_steps:
        b.set_graphs(False)
        b.prefetch_prologue(grads_only=world > 1)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with DP.capture(g):
            for _ in range(graph_steps):
                step(b, True)
        for _ in range(6 // graph_steps):
            g.replay()
        C_ = __import__("dqn._capi", fromlist=["lib"])
        C_.check(C_.lib().dqnx_prefetch_stream(b.h, b.stream()), "prefetch_stream")
    else:
        for _ in range(6):
            step(b, True)
    step(b, False)   # consumes the pending draw
    torch.cuda.synchronize()
    b.check_device_error()
    assert torch.equal(a.batch_idx, b.batch_idx)
    assert np.array_equal(a.get_rng(0), b.get_rng(0))
    assert torch.equal(a.params, b.params)
    assert torch.equal(a.target_params, b.target_params)
