"""GPU: the acting path (`dqnx_act`, one launch per Network.actions call) against the oracle's
torch-CPU forward (R:dqn/network.py:67-74 DeepQNetwork, :110-117 Dueling: advantage argmax).

Values within 1e-5 (scaled by max(1, |v|)); actions equal the oracle's argmax wherever the
top-two gap exceeds that tolerance (closer ties are decided by summation order, which no
fp32 implementation shares with torch's CPU GEMM)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from dqn import engine as E
from dqn.network import DeepQNetwork, DuelingDeepQNetwork
from oracle import ref as O
from refnets import Box, mlp_network_config

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _flat(espec, params):
    n, layout = espec.param_infos()
    flat = torch.empty(n, dtype=torch.float32)
    for name, off, shape in layout:
        flat[off:off + int(np.prod(shape))] = params[name].reshape(-1)
    return flat.cuda()


def _check(vals, ref, acts):
    np.testing.assert_allclose(vals, ref, atol=TOL * max(1.0, float(np.abs(ref).max())), rtol=0)
    srt = np.sort(ref, axis=1)
    clear = (srt[:, -1] - srt[:, -2]) > 4 * TOL * max(1.0, float(np.abs(ref).max()))
    assert np.array_equal(acts[clear], ref.argmax(axis=1)[clear])
    assert clear.mean() > 0.9


@pytest.mark.parametrize("obs_dim", [14, 284])
@pytest.mark.parametrize("head", ["dueling", "linear"])
@pytest.mark.parametrize("n", [1, 2, 3, 8, 37, 1000])
def test_gpu_act_matches_oracle(obs_dim, head, n):
    ospec = O.mlp_spec(obs_dim, 8, head)
    params = O.reference_init(ospec, 5)
    espec = E.mlp_spec(obs_dim, 8, head)
    flat = _flat(espec, params)
    x = torch.from_numpy(np.random.default_rng(n).random((n, obs_dim), dtype=np.float32))
    vals = torch.empty(n, 8, dtype=torch.float32, device="cuda")
    acts = E.act(espec, flat, x.cuda(), vals)
    torch.cuda.synchronize()
    with torch.no_grad():
        ref = (O.advantages(ospec, params, x) if head == "dueling" else O.q_forward(ospec, params, x)).numpy()
    _check(vals.cpu().numpy(), ref, acts.cpu().numpy())


def test_gpu_act_elu_deep_wide_body():
    """ELU body, 3 layers up to 600 wide, odd action count: the generic layer loop."""
    spec = E.NetSpec(kind=E.C.DQNX_NET_MLP, head=E.C.DQNX_HEAD_LINEAR, activation=E.C.DQNX_ACT_ELU,
                     obs_dim=37, n_actions=5, dense=(600, 130, 64))
    n_params, layout = spec.param_infos()
    g = torch.Generator().manual_seed(0)
    flat = torch.randn(n_params, generator=g) * 0.2
    P = {name: flat[off:off + int(np.prod(s))].view(*s) for name, off, s in layout}
    x = torch.randn(9, 37, generator=g)
    h = x
    for l in range(3):
        h = F.elu(F.linear(h, P[f"net.{2 * l}.weight"], P[f"net.{2 * l}.bias"]))
    ref = F.linear(h, P["fc_out.weight"], P["fc_out.bias"]).numpy()
    vals = torch.empty(9, 5, device="cuda")
    acts = E.act(spec, flat.cuda(), x.cuda(), vals)
    _check(vals.cpu().numpy(), ref, acts.cpu().numpy())


def test_gpu_act_shared_scratch_across_row_counts():
    """One scratch serves calls with different n in any order (tickets never clobbered)."""
    ospec = O.mlp_spec(284, 8, "dueling")
    params = O.reference_init(ospec, 6)
    espec = E.mlp_spec(284, 8, "dueling")
    flat = _flat(espec, params)
    scratch = E.act_scratch(espec, 64, "cuda")
    rng = np.random.default_rng(0)
    for n in (64, 1, 3, 2, 64, 5, 1, 33):
        x = torch.from_numpy(rng.random((n, 284), dtype=np.float32))
        vals = torch.empty(n, 8, device="cuda")
        acts = E.act(espec, flat, x.cuda(), vals, scratch=scratch)
        with torch.no_grad():
            ref = O.advantages(ospec, params, x).numpy()
        _check(vals.cpu().numpy(), ref, acts.cpu().numpy())


@pytest.mark.parametrize("head", ["dueling", "linear"])
@pytest.mark.parametrize("n", [1, 2, 3, 8, 37])
def test_gpu_act_two_stream_matches_oracle(head, n):
    """The reference's HEAD network (TwoStreamHybridNetwork on the 2x27x5 grid, R:env/dqn_config.py
    :66-193): conv launches + the MLP acting kernel on cat(flatten(conv3), macro)."""
    ospec = O.hybrid_spec(8, head)
    params = O.reference_init(ospec, 7)
    espec = E.hybrid_spec(8, head)
    flat = _flat(espec, params)
    x = torch.from_numpy(O.synth_transitions(n, ospec.obs_dim, 8, seed=n)[0])
    vals = torch.empty(n, 8, dtype=torch.float32, device="cuda")
    acts = E.act(espec, flat, x.cuda(), vals)
    torch.cuda.synchronize()
    with torch.no_grad():
        ref = (O.advantages(ospec, params, x) if head == "dueling" else O.q_forward(ospec, params, x)).numpy()
    _check(vals.cpu().numpy(), ref, acts.cpu().numpy())


def test_gpu_act_two_stream_84_falls_back():
    """The (4,84,84) variant's conv input does not fit the acting kernel: dqnx_act refuses it and
    Network.actions keeps the torch forward."""
    spec = E.hybrid_spec(micro_chw=(4, 84, 84))
    assert not E.act_supported(spec)
    assert E.act_supported(E.hybrid_spec())


@pytest.mark.parametrize("cls", [DeepQNetwork, DuelingDeepQNetwork])
def test_gpu_standalone_two_stream_network_actions(cls):
    """Observe-style use of the HEAD net: a standalone two-stream network acts through dqnx_act."""
    from refnets import hybrid_network_config
    torch.manual_seed(5)
    net = cls("cuda:0", 1e-4, hybrid_network_config, Box(284), 8)
    x = O.synth_transitions(6, 284, 8, seed=2)[0]
    xt = torch.from_numpy(x).cuda()
    assert net._native_act() is not None
    with torch.no_grad():
        q = (net.advantages(xt) if cls is DuelingDeepQNetwork else net(xt)).cpu().numpy()
    got = net.actions(x)
    srt = np.sort(q, axis=1)
    clear = (srt[:, -1] - srt[:, -2]) > 1e-4
    assert np.array_equal(np.asarray(got)[clear], q.argmax(1)[clear])


@pytest.mark.parametrize("cls", [DeepQNetwork, DuelingDeepQNetwork])
def test_gpu_standalone_network_actions(cls):
    """Observe-style use (R:observe.py:24-37): a network built on its own, then reloaded."""
    torch.manual_seed(3)
    net = cls("cuda:0", 1e-4, mlp_network_config, Box(284), 8)
    x = np.random.default_rng(1).random((4, 284), dtype=np.float32)
    xt = torch.from_numpy(x).cuda()
    with torch.no_grad():
        ref = (net.advantages(xt) if cls is DuelingDeepQNetwork else net(xt)).argmax(1).tolist()
    assert net.actions(x) == ref
    # new weights through load_state_dict land in the kernel's buffer
    torch.manual_seed(4)
    other = cls("cuda:0", 1e-4, mlp_network_config, Box(284), 8)
    net.load_state_dict(other.state_dict())
    with torch.no_grad():
        ref2 = (other.advantages(xt) if cls is DuelingDeepQNetwork else other(xt)).argmax(1).tolist()
    assert net.actions(x) == ref2


@pytest.mark.parametrize("net", ["mlp", "two_stream"])
def test_gpu_act_host_shared_scratch_across_row_counts(net):
    """dqnx_act_host with one scratch buffer and n = 64 then smaller n: the acting kernel's
    arrival tickets must sit at the same address for every n.  They used to follow the end of the
    n-dependent acting region, and on the two-stream path a 64-row call's obs filled the words an
    8-row call then took for its tickets: its last-arriver test never fired and stale actions came
    back without an error.  Every call's actions and values are compared with dqnx_act's."""
    import ctypes

    from dqn import _capi as C
    if net == "mlp":
        ospec, espec = O.mlp_spec(284, 8, "dueling"), E.mlp_spec(284, 8, "dueling")
    else:
        ospec, espec = O.hybrid_spec(8, "dueling"), E.hybrid_spec(8, "dueling")
    params = O.reference_init(ospec, 8)
    flat = _flat(espec, params)
    desc = espec.to_c()
    L = C.lib()
    nb = int(L.dqnx_act_host_scratch_bytes(ctypes.byref(desc), 64))
    scratch = torch.zeros((nb + 15) // 16 * 4, dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for n in (64, 8, 1, 64, 3, 8):
        x = O.synth_transitions(n, ospec.obs_dim, 8, seed=100 + n)[0]
        x = np.ascontiguousarray(x, dtype=np.float32) + np.float32(0.25)   # obs words far from 0
        out = np.full(n, -1, dtype=np.int32)
        C.check(L.dqnx_act_host(ctypes.byref(desc), flat.data_ptr(), x.ctypes.data, n, out.ctypes.data,
                                scratch.data_ptr(), scratch.numel() * 4, stream), "act_host")
        vals = torch.empty(n, 8, dtype=torch.float32, device="cuda")
        acts = E.act(espec, flat, torch.from_numpy(x).cuda(), vals).cpu().numpy()
        assert np.array_equal(out, acts), (n, out, acts)
        with torch.no_grad():
            ref = O.advantages(ospec, params, torch.from_numpy(x)).numpy()
        _check(vals.cpu().numpy(), ref, out)


@pytest.mark.parametrize("G", ["1", "2", "4", "8"])
@pytest.mark.parametrize("head", ["dueling", "linear"])
@pytest.mark.parametrize("n", [1, 2])
def test_gpu_act_one_round_trip_kernel_workgroups(monkeypatch, G, head, n):
    """k_act_mlp1 with its layer-1 neurons over G workgroups (DQNX_ACT1_G; layer-2 shares summed by the
    last arriving workgroup after a write-through hand-off) against the oracle, through dqnx_act_host
    (the agent's path, completion word polled) and dqnx_act; repeated calls reuse the arrival ticket."""
    import ctypes

    from dqn import _capi as C
    monkeypatch.setenv("DQNX_ACT1_G", G)
    ospec, espec = O.mlp_spec(284, 8, head), E.mlp_spec(284, 8, head)
    params = O.reference_init(ospec, 21)
    flat = _flat(espec, params)
    desc = espec.to_c()
    L = C.lib()
    nb = int(L.dqnx_act_host_scratch_bytes(ctypes.byref(desc), n))
    scratch = torch.zeros((nb + 15) // 16 * 4, dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for rep in range(6):
        x = np.ascontiguousarray(np.random.default_rng(100 * rep + n).random((n, 284), dtype=np.float32))
        out = np.full(n, -1, dtype=np.int32)
        C.check(L.dqnx_act_host(ctypes.byref(desc), flat.data_ptr(), x.ctypes.data, n, out.ctypes.data,
                                scratch.data_ptr(), scratch.numel() * 4, stream), "act_host")
        vals = torch.empty(n, 8, dtype=torch.float32, device="cuda")
        acts = E.act(espec, flat, torch.from_numpy(x).cuda(), vals).cpu().numpy()
        assert np.array_equal(out, acts), (rep, out, acts)
        with torch.no_grad():
            xt = torch.from_numpy(x)
            ref = (O.advantages(ospec, params, xt) if head == "dueling" else O.q_forward(ospec, params, xt)).numpy()
        _check(vals.cpu().numpy(), ref, out)


@pytest.mark.parametrize("obs_dim,n", [(3000, 3), (3000, 2), (5000, 2), (5000, 1)])
def test_gpu_act_host_wide_inputs_several_row_groups(obs_dim, n):
    """dqnx_act_host on inputs wider than 2048 / 4096 floats, where a workgroup takes 2 / 1 rows:
    a launch with several row groups stores no completion word, so the call must not poll for one (it
    used to spin 0.5 s per call before falling back to a stream synchronize).  Actions equal dqnx_act's,
    and 20 calls finish well inside one poll timeout."""
    import ctypes
    import time

    from dqn import _capi as C
    ospec, espec = O.mlp_spec(obs_dim, 8, "dueling"), E.mlp_spec(obs_dim, 8, "dueling")
    params = O.reference_init(ospec, 8)
    flat = _flat(espec, params)
    desc = espec.to_c()
    L = C.lib()
    nb = int(L.dqnx_act_host_scratch_bytes(ctypes.byref(desc), n))
    scratch = torch.zeros((nb + 15) // 16 * 4, dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    x = np.ascontiguousarray(np.random.default_rng(obs_dim + n).random((n, obs_dim), dtype=np.float32))
    out = np.full(n, -1, dtype=np.int32)
    C.check(L.dqnx_act_host(ctypes.byref(desc), flat.data_ptr(), x.ctypes.data, n, out.ctypes.data,
                            scratch.data_ptr(), scratch.numel() * 4, stream), "act_host")
    vals = torch.empty(n, 8, dtype=torch.float32, device="cuda")
    acts = E.act(espec, flat, torch.from_numpy(x).cuda(), vals).cpu().numpy()
    assert np.array_equal(out, acts), (out, acts)
    t0 = time.perf_counter()
    for _ in range(20):
        C.check(L.dqnx_act_host(ctypes.byref(desc), flat.data_ptr(), x.ctypes.data, n, out.ctypes.data,
                                scratch.data_ptr(), scratch.numel() * 4, stream), "act_host")
    assert time.perf_counter() - t0 < 0.4, "act_host waited for a completion word its launch never stores"
    assert np.array_equal(out, acts)


@pytest.mark.parametrize("kernel", ["0", "1"])
@pytest.mark.parametrize("head", ["dueling", "linear"])
@pytest.mark.parametrize("n", [1, 2, 5, 64])
def test_gpu_act_two_hidden_layer_kernels(monkeypatch, kernel, head, n):
    """Both acting kernels of a two-hidden-layer MLP against the oracle: k_act_mlp (DQNX_ACT2=0: the last
    workgroup runs layer 2 on the gathered h1) and k_act_mlp2 (the default: layer 2 summed from the
    layer-1 workgroups' shares, its weights and the head's fetched at the top of the kernel)."""
    monkeypatch.setenv("DQNX_ACT2", kernel)
    ospec = O.mlp_spec(284, 8, head)
    params = O.reference_init(ospec, 9)
    espec = E.mlp_spec(284, 8, head)
    flat = _flat(espec, params)
    x = torch.from_numpy(np.random.default_rng(100 + n).random((n, 284), dtype=np.float32))
    scratch = E.act_scratch(espec, 64, "cuda")
    for _ in range(3):   # the same scratch (tickets) across calls
        vals = torch.empty(n, 8, dtype=torch.float32, device="cuda")
        acts = E.act(espec, flat, x.cuda(), vals, scratch=scratch)
        torch.cuda.synchronize()
        with torch.no_grad():
            ref = (O.advantages(ospec, params, x) if head == "dueling" else O.q_forward(ospec, params, x)).numpy()
        _check(vals.cpu().numpy(), ref, acts.cpu().numpy())
