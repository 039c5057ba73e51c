"""CPU checks of the C ABI (include/dqnx.h <-> libdqnx.so <-> dqn/_capi.py).

No GPU calls: the library must load, export every entry point the header declares,
agree with gcc on every struct layout, and plan parameter tables whose names / shapes /
counts equal the reference networks' state_dict (R:dqn/network.py, R:env/dqn_config.py).
"""
import ctypes
import os
import re
import subprocess

import pytest

from dqn import _capi as C
from oracle import ref as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "dqnx.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dqnx_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = C.lib()
    declared = header_functions()
    assert declared, "no declarations parsed"
    missing = [f for f in declared if not hasattr(L, f)]
    assert not missing, missing
    assert sorted(C.EXPORTS) == declared, set(C.EXPORTS) ^ set(declared)


def test_abi_version_matches_header():
    m = re.search(r"#define\s+DQNX_ABI_VERSION\s+(\d+)", open(HEADER).read())
    assert m and C.lib().dqnx_abi_version() == int(m.group(1))


def _gcc_layout(tmp_path):
    prog = tmp_path / "layout.c"
    structs = {
        "dqnx_net_desc": C.NetDesc, "dqnx_param_info": C.ParamInfo,
        "dqnx_config": C.Config, "dqnx_ctrl": C.Ctrl,
    }
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines += ["return 0;", "}"]
    prog.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c11", "-o", str(exe), str(prog)])
    out = subprocess.check_output([str(exe)]).decode().split("\n")
    return structs, [ln.split() for ln in out if ln]


def test_struct_layouts_match_gcc(tmp_path):
    structs, rows = _gcc_layout(tmp_path)
    for cname, field, val in rows:
        py = structs[cname]
        got = ctypes.sizeof(py) if field == "sizeof" else getattr(py, field).offset
        assert got == int(val), (cname, field, got, val)


def _engine_spec(ospec):
    from dqn import engine as E
    if ospec.kind == "mlp":
        return E.mlp_spec(ospec.obs_dim, ospec.n_actions, ospec.head, ospec.hidden)
    return E.NetSpec(kind=C.DQNX_NET_TWO_STREAM,
                     head=C.DQNX_HEAD_DUELING if ospec.head == "dueling" else C.DQNX_HEAD_LINEAR,
                     activation=C.DQNX_ACT_ELU, obs_dim=ospec.obs_dim, n_actions=ospec.n_actions,
                     dense=tuple(ospec.dense), macro_len=ospec.macro_len, micro_chw=tuple(ospec.micro_chw),
                     conv=tuple(ospec.conv))


@pytest.mark.parametrize("ospec,expected", [
    (O.mlp_spec(284, 8, "dueling"), 107017),     # SURVEY.md section 8 counts
    (O.mlp_spec(284, 8, "linear"), None),
    (O.mlp_spec(14, 8, "dueling"), None),
    (O.hybrid_spec(8, "dueling"), 885481),
    (O.hybrid_spec(8, "linear"), None),
])
def test_param_tables_match_reference_networks(ospec, expected):
    total, infos = _engine_spec(ospec).param_infos()
    ref = O.reference_init(ospec, 0)
    assert [i[0] for i in infos] == list(ref.keys())
    off = 0
    for (name, offset, shape), t in zip(infos, ref.values()):
        assert tuple(shape) == tuple(t.shape), name
        assert offset == off, name          # flat, contiguous, state_dict order
        off += t.numel()
    assert total == off
    if expected is not None:
        assert total == expected


def test_config_defaults_follow_reference_agent():
    cfg = C.Config()
    C.lib().dqnx_config_defaults(ctypes.byref(cfg))
    # R:dqn/agent.py Agent.__init__ defaults / torch.optim.Adam defaults
    assert cfg.beta1 == 0.9 and cfg.beta2 == 0.999 and cfg.adam_eps == 1e-8
    assert cfg.world_size == 1 and cfg.rank == 0


def test_engine_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from dqn import engine as E
    with pytest.raises(RuntimeError):
        E.LearnEngine(E.mlp_spec(14, 8, "dueling"), "DuelingDoubleDQNAgent", 32, 500)


def _create(spec, dtype):
    cfg = C.Config()
    cfg.net = spec.to_c()
    C.lib().dqnx_config_defaults(ctypes.byref(cfg))
    cfg.batch, cfg.capacity = 64, 1000
    cfg.compute_dtype = dtype
    h = ctypes.c_void_p()
    rc = C.lib().dqnx_engine_create(ctypes.byref(cfg), ctypes.byref(h))
    if rc == 0:
        C.lib().dqnx_engine_destroy(h)
    return rc


def test_bf16_compute_is_mlp_only():
    """bf16 lives in the fused MLP kernels; other nets and unknown dtypes are refused at create."""
    from dqn import engine as E
    assert _create(E.mlp_spec(284, 8, "dueling"), C.DQNX_COMPUTE_BF16) == 0
    assert _create(E.mlp_spec(14, 8, "linear"), C.DQNX_COMPUTE_BF16) == 0
    assert _create(_engine_spec(O.hybrid_spec(8, "dueling")), C.DQNX_COMPUTE_BF16) == C.DQNX_EUNSUPPORTED
    assert _create(E.mlp_spec(284, 8, "dueling"), 7) == C.DQNX_EINVAL


def test_act_argument_checks_without_gpu():
    """dqnx_act validates on the host before any launch: two-stream nets are refused,
    null buffers rejected, n = 0 is a no-op."""
    from dqn import engine as E
    L = C.lib()
    hyb = _engine_spec(O.hybrid_spec(8, "dueling")).to_c()
    mlp = E.mlp_spec(284, 8, "dueling").to_c()
    need_h = L.dqnx_act_scratch_bytes(ctypes.byref(hyb), 1)
    assert need_h > 0   # two-stream nets act too (conv launches + the MLP acting kernel)
    assert L.dqnx_act(ctypes.byref(hyb), 16, 16, 1, 16, None, 16, need_h - 4, None) == C.DQNX_EINVAL
    assert L.dqnx_act(ctypes.byref(mlp), None, None, 4, None, None, None, 0, None) == C.DQNX_EINVAL
    assert L.dqnx_act(ctypes.byref(mlp), None, None, 0, None, None, None, 0, None) == C.DQNX_OK
    need = L.dqnx_act_scratch_bytes(ctypes.byref(mlp), 3)
    # one group of R = 4 rows: the larger of k_act_mlp's layer-1 activations [4][256] and k_act_mlp2's
    # layer-2 shares [16 workgroups][4][128], + its ticket
    assert need == max(4 * 256, 16 * 4 * 128) * 4 + 4
    # too small a scratch is refused before any launch
    assert L.dqnx_act(ctypes.byref(mlp), 16, 16, 3, 16, None, 16, need - 4, None) == C.DQNX_EINVAL
