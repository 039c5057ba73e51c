"""LearnEngine: the Python face of libdqnx (one engine = one agent's learn-step state).

The engine's whole device state lives in ONE torch-allocated HBM arena (parameters,
target parameters, gradient, Adam moments, control block, replay ring, workspace);
libdqnx only borrows it.  ``LearnEngine`` exposes torch views of every region so the
host shim can keep the reference's ``state_dict()`` / checkpoint behaviour.

No CPU fallback: constructing an engine without a GPU or without libdqnx.so raises.
"""
from __future__ import annotations

import ctypes
import random
import struct
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn

from . import _capi as C

ALGO_IDS = {"DQNAgent": C.DQNX_ALGO_DQN, "DoubleDQNAgent": C.DQNX_ALGO_DOUBLE,
            "DuelingDoubleDQNAgent": C.DQNX_ALGO_DOUBLE, "PerDuelingDoubleDQNAgent": C.DQNX_ALGO_PER_DOUBLE}


# ----------------------------------------------------------------------------------------
# network description
# ----------------------------------------------------------------------------------------
@dataclass
class NetSpec:
    """What libdqnx needs to know about a Q-network (mirrors dqnx_net_desc)."""
    kind: int = C.DQNX_NET_MLP
    head: int = C.DQNX_HEAD_DUELING
    activation: int = C.DQNX_ACT_RELU
    obs_dim: int = 284
    n_actions: int = 8
    dense: Tuple[int, ...] = (256, 128)
    macro_len: int = 0
    micro_chw: Tuple[int, int, int] = (0, 0, 0)
    conv: Tuple[Tuple[int, Tuple[int, int], Tuple[int, int]], ...] = ()

    def to_c(self) -> C.NetDesc:
        d = C.NetDesc()
        d.kind, d.head, d.activation = self.kind, self.head, self.activation
        d.obs_dim, d.n_actions = self.obs_dim, self.n_actions
        d.n_dense = len(self.dense)
        for i, w in enumerate(self.dense):
            d.dense[i] = w
        d.macro_len = self.macro_len
        d.micro_c, d.micro_h, d.micro_w = self.micro_chw
        d.n_conv = len(self.conv)
        for i, (f, (kh, kw), (sh, sw)) in enumerate(self.conv):
            d.conv_out[i], d.conv_kh[i], d.conv_kw[i], d.conv_sh[i], d.conv_sw[i] = f, kh, kw, sh, sw
        return d

    def param_infos(self):
        L = C.lib()
        d = self.to_c()
        n = C.I64()
        nt = C.I32()
        C.check(L.dqnx_net_param_count(ctypes.byref(d), ctypes.byref(n), ctypes.byref(nt)), "param_count")
        out = []
        for i in range(nt.value):
            pi = C.ParamInfo()
            C.check(L.dqnx_net_param_info(ctypes.byref(d), i, ctypes.byref(pi)), "param_info")
            out.append((pi.name.decode(), int(pi.offset), tuple(pi.shape[:pi.ndim])))
        return int(n.value), out


def mlp_spec(obs_dim=284, n_actions=8, head="dueling", hidden=(256, 128)) -> NetSpec:
    return NetSpec(kind=C.DQNX_NET_MLP, head=C.DQNX_HEAD_DUELING if head == "dueling" else C.DQNX_HEAD_LINEAR,
                   activation=C.DQNX_ACT_RELU, obs_dim=obs_dim, n_actions=n_actions, dense=tuple(hidden))


HYBRID_CONV = ((32, (3, 3), (1, 1)), (64, (3, 3), (2, 1)), (64, (3, 3), (2, 2)))   # R:env/dqn_config.py:163-167


def hybrid_spec(n_actions=8, head="dueling", micro_chw=(2, 27, 5), macro_len=14, conv=HYBRID_CONV,
                dense=(512, 256)) -> NetSpec:
    """TwoStreamHybridNetwork as network_config builds it (R:env/dqn_config.py:148-193)."""
    c, h, w = micro_chw
    return NetSpec(kind=C.DQNX_NET_TWO_STREAM, head=C.DQNX_HEAD_DUELING if head == "dueling" else C.DQNX_HEAD_LINEAR,
                   activation=C.DQNX_ACT_ELU, obs_dim=macro_len + c * h * w, n_actions=n_actions,
                   dense=tuple(dense), macro_len=macro_len, micro_chw=tuple(micro_chw), conv=tuple(conv))


def spec_from_body(net: nn.Module, obs_dim: int, n_actions: int, dueling: bool) -> NetSpec:
    """Recognise the two body families the reference ships (SURVEY §7 hard part 6) and
    refuse anything else:
      * nn.Sequential(Linear, ReLU|ELU, Linear, ReLU|ELU, ...)
        (R:env/custom_env/macro with lane/dqn_config.py:76-84)
      * TwoStreamHybridNetwork (R:env/dqn_config.py:66-143)."""
    head = C.DQNX_HEAD_DUELING if dueling else C.DQNX_HEAD_LINEAR
    if isinstance(net, nn.Sequential):
        mods = list(net)
        if len(mods) % 2 or len(mods) == 0:
            raise NotImplementedError("libdqnx: MLP body must alternate Linear and activation")
        dense, act = [], None
        d = obs_dim
        for i in range(0, len(mods), 2):
            lin, a = mods[i], mods[i + 1]
            if not isinstance(lin, nn.Linear) or lin.in_features != d or lin.bias is None:
                raise NotImplementedError(f"libdqnx: unsupported MLP layer {lin!r}")
            k = C.DQNX_ACT_RELU if isinstance(a, nn.ReLU) else (C.DQNX_ACT_ELU if isinstance(a, nn.ELU) else None)
            if k is None or (act is not None and k != act):
                raise NotImplementedError(f"libdqnx: unsupported activation {a!r}")
            if isinstance(a, nn.ELU) and a.alpha != 1.0:
                raise NotImplementedError("libdqnx: ELU alpha must be 1")
            act = k
            dense.append(lin.out_features)
            d = lin.out_features
        return NetSpec(kind=C.DQNX_NET_MLP, head=head, activation=act, obs_dim=obs_dim, n_actions=n_actions,
                       dense=tuple(dense))
    if hasattr(net, "cnn_stream") and hasattr(net, "dense_stream") and hasattr(net, "micro_shape"):
        # TwoStreamHybridNetwork (R:env/dqn_config.py:66-143): [Conv2d, act]* then [Linear, act]*;
        # the engine plans exactly that layer sequence, so refuse anything it would plan differently
        conv = []
        mods = list(net.cnn_stream)
        c, h, w = (int(x) for x in net.micro_shape)
        macro_len = int(net.macro_len)
        if len(mods) % 2 or not mods:
            raise NotImplementedError("libdqnx: cnn_stream must alternate Conv2d and activation")
        for i in range(0, len(mods), 2):
            cv = mods[i]
            ok = (isinstance(cv, nn.Conv2d) and cv.in_channels == c and cv.bias is not None
                  and cv.padding == (cv.kernel_size[0] // 2, cv.kernel_size[1] // 2)
                  and tuple(cv.dilation) == (1, 1) and cv.groups == 1 and cv.padding_mode == "zeros")
            if not ok:
                raise NotImplementedError(f"libdqnx: unsupported conv {cv!r}")
            (kh, kw), (sh, sw) = tuple(cv.kernel_size), tuple(cv.stride)
            h = (h + 2 * (kh // 2) - kh) // sh + 1
            w = (w + 2 * (kw // 2) - kw) // sw + 1
            c = cv.out_channels
            conv.append((cv.out_channels, (kh, kw), (sh, sw)))
        dmods = list(net.dense_stream)
        if len(dmods) % 2 or not dmods:
            raise NotImplementedError("libdqnx: dense_stream must alternate Linear and activation")
        dense = []
        d = c * h * w + macro_len      # flatten(conv) ++ macro (R:env/dqn_config.py:135-138)
        for i in range(0, len(dmods), 2):
            lin = dmods[i]
            if not isinstance(lin, nn.Linear) or lin.in_features != d or lin.bias is None:
                raise NotImplementedError(f"libdqnx: unsupported dense layer {lin!r} (expects in_features {d})")
            dense.append(lin.out_features)
            d = lin.out_features
        acts = mods[1::2] + dmods[1::2]
        if not all(isinstance(a, nn.ELU) and a.alpha == 1.0 for a in acts):
            raise NotImplementedError("libdqnx: two-stream net must use ELU(alpha=1)")
        cm, hm, wm = (int(x) for x in net.micro_shape)
        if obs_dim != macro_len + cm * hm * wm:
            raise NotImplementedError(f"libdqnx: obs_dim {obs_dim} != macro_len + prod(micro_shape)")
        return NetSpec(kind=C.DQNX_NET_TWO_STREAM, head=head, activation=C.DQNX_ACT_ELU, obs_dim=obs_dim,
                       n_actions=n_actions, dense=tuple(dense), macro_len=macro_len,
                       micro_chw=(cm, hm, wm), conv=tuple(conv))
    raise NotImplementedError(f"libdqnx: unsupported Q-network body {type(net).__name__}")


# ----------------------------------------------------------------------------------------
# acting path (dqnx_act)
# ----------------------------------------------------------------------------------------
def act_scratch(spec: NetSpec, n: int, device) -> torch.Tensor:
    """Zeroed scratch for dqnx_act calls of up to n rows (reusable across calls on one stream)."""
    nbytes = int(C.lib().dqnx_act_scratch_bytes(ctypes.byref(spec.to_c()), int(n)))
    return torch.zeros((nbytes + 15) // 16 * 4, dtype=torch.float32, device=device)


def act_supported(spec: NetSpec) -> bool:
    """dqnx_act implements this network (MLP bodies; two-stream bodies whose conv inputs fit the
    acting kernel's LDS, e.g. the reference's 2x27x5 grid but not the 4x84x84 variant)."""
    return int(C.lib().dqnx_act_scratch_bytes(ctypes.byref(spec.to_c()), 1)) > 0


def act(spec: NetSpec, flat: torch.Tensor, obs: torch.Tensor, values: Optional[torch.Tensor] = None,
        scratch: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None, desc=None) -> torch.Tensor:
    """Greedy actions of a Q-network on the GPU (`dqnx_act`: one launch for an MLP, the conv
    launches + the MLP kernel for a two-stream net).

    `flat`: the network's flat fp32 parameters on the GPU (dqnx_net_param_info layout);
    `obs`: [n, obs_dim] on the same GPU.  Returns int32 actions [n] (first maximal index, like
    torch.argmax) of Q, or of the advantage stream for a dueling head (R:dqn/network.py:67-74,
    110-117).  `values`, if given ([n, n_actions] fp32), receives the argmaxed values."""
    obs = obs.to(flat.device, torch.float32).contiguous()
    if obs.dim() != 2 or obs.shape[1] != spec.obs_dim:
        raise ValueError(f"obs must be [n, {spec.obs_dim}], got {tuple(obs.shape)}")
    n = obs.shape[0]
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=flat.device)
    elif out.dtype != torch.int32 or out.device != flat.device or out.numel() < n or not out.is_contiguous():
        raise ValueError("out must be a contiguous int32 tensor of >= n elements on the parameters' device")
    if values is not None and (values.shape != (n, spec.n_actions) or not values.is_contiguous()
                               or values.dtype != torch.float32 or values.device != flat.device):
        raise ValueError("values must be a contiguous fp32 [n, n_actions] tensor on the parameters' device")
    if scratch is None:
        scratch = act_scratch(spec, n, flat.device)
    d = spec.to_c() if desc is None else desc
    stream = ctypes.c_void_p(torch.cuda.current_stream(flat.device).cuda_stream)
    C.check(C.lib().dqnx_act(ctypes.byref(d), flat.data_ptr(), obs.data_ptr(), n, out.data_ptr(),
                             values.data_ptr() if values is not None else None, scratch.data_ptr(),
                             scratch.numel() * 4, stream), "act")
    return out[:n]


# ----------------------------------------------------------------------------------------
# engine
# ----------------------------------------------------------------------------------------
class LearnEngine:
    """One agent's learn-step engine on one GPU (one process per GPU under DP)."""

    def __init__(self, spec: NetSpec, algo: str, batch: int, capacity: int, gamma=0.99, lr=1e-4,
                 tau=1e-3, n_env=1, world_size=1, rank=0, device=None, graphs=False, eps_dec=2e6,
                 local_sampling=False, compute_dtype="fp32", per_numpy121=False):
        """graphs: replay each learn step as a captured HIP graph (off by default: eager launches
        measured 3-4 us faster per step, include/dqnx.h dqnx_engine_set_graphs).
        per_numpy121: PER SumTree arithmetic of the reference's pinned numpy 1.21 (float32
        `change` and float32-rounded ancestor sums, in update order) instead of numpy >= 2's."""
        if not torch.cuda.is_available():
            raise RuntimeError("libdqnx needs a ROCm GPU (MI355X / gfx950); there is no CPU fallback")
        self.L = C.lib()
        self.spec = spec
        self.algo = algo
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        cfg = C.Config()
        cfg.net = spec.to_c()
        self.L.dqnx_config_defaults(ctypes.byref(cfg))
        cfg.algo = ALGO_IDS[algo] if isinstance(algo, str) else int(algo)
        cfg.batch, cfg.world_size, cfg.rank, cfg.capacity = batch, world_size, rank, capacity
        cfg.gamma, cfg.lr, cfg.tau, cfg.n_env = gamma, lr, tau, n_env
        cfg.per_beta_steps = eps_dec
        cfg.local_sampling = 1 if local_sampling else 0
        if compute_dtype not in ("fp32", "bf16"):
            raise ValueError(f"compute_dtype must be 'fp32' or 'bf16', got {compute_dtype!r}")
        cfg.compute_dtype = C.DQNX_COMPUTE_BF16 if compute_dtype == "bf16" else C.DQNX_COMPUTE_FP32
        cfg.per_numpy121 = 1 if per_numpy121 else 0
        self.compute_dtype = compute_dtype
        self.cfg = cfg
        h = ctypes.c_void_p()
        C.check(self.L.dqnx_engine_create(ctypes.byref(cfg), ctypes.byref(h)), "dqnx_engine_create")
        self.h = h
        self._ag_unread = False   # an agent step's control-block readback not yet consumed
        nbytes = ctypes.c_uint64()
        C.check(self.L.dqnx_engine_arena_bytes(h, ctypes.byref(nbytes)), "arena_bytes")
        self.arena = torch.zeros(int(nbytes.value), dtype=torch.uint8, device=self.device)
        C.check(self.L.dqnx_engine_bind(h, ctypes.c_void_p(self.arena.data_ptr()), nbytes.value), "bind")
        C.check(self.L.dqnx_engine_set_graphs(h, 1 if graphs else 0), "set_graphs")
        st = C.I32()
        C.check(self.L.dqnx_engine_obs_stride(h, ctypes.byref(st)), "obs_stride")
        self.obs_stride = st.value
        self.batch, self.capacity, self.world_size, self.rank = batch, capacity, world_size, rank
        self.batch_local = batch // world_size
        self.n_params, self.param_layout = spec.param_infos()
        self.reset()
        self.params = self.view(C.BUF_PARAMS, torch.float32)
        self.target_params = self.view(C.BUF_TARGET_PARAMS, torch.float32)
        self.grads = self.view(C.BUF_GRADS, torch.float32)          # [P + 1], last = loss
        self.adam_m = self.view(C.BUF_ADAM_M, torch.float32)
        self.adam_v = self.view(C.BUF_ADAM_V, torch.float32)
        self.ctrl_bytes = self.view(C.BUF_CTRL, torch.uint8)
        self.batch_idx_slots = self.view(C.BUF_BATCH_IDX, torch.int32).view(2, batch)
        self.batch_idx = self.batch_idx_slots[0]
        self.q = self.view(C.BUF_Q, torch.float32).view(3, self.batch_local, spec.n_actions)
        self.td = self.view(C.BUF_TD, torch.float32).view(3, self.batch_local)
        self.is_weights = self.view(C.BUF_IS_WEIGHTS, torch.float32)
        self.ring_obs = self.view(C.BUF_RING_OBS, torch.float32).view(capacity, self.obs_stride)
        self.ring_next_obs = self.view(C.BUF_RING_NEXT_OBS, torch.float32).view(capacity, self.obs_stride)
        self.ring_act = self.view(C.BUF_RING_ACT, torch.int32)
        self.ring_rew = self.view(C.BUF_RING_REW, torch.float32)
        self.ring_done = self.view(C.BUF_RING_DONE, torch.float32)
        self.sumtree = self.view(C.BUF_SUMTREE, torch.float64)      # [2*cap-1] (PER), else empty
        self.per_abs_td = self.view(C.BUF_PER_ABS_TD, torch.float32)  # [batch] (PER), else empty
        self.ring_size = 0
        self.ring_wptr = 0
        self.agent_step = 0      # host mirror of dqnx_ctrl.agent_step (PER beta schedule)
        # set by a drop-in Agent that records learn() steps for launch at its next call: `launch_hook`
        # launches a recorded step (host reads of engine memory follow it in stream order),
        # `settle_hook` also waits for it and raises a device error it reported
        self.launch_hook = None
        self.settle_hook = None

    def launch_recorded(self):
        if self.launch_hook is not None:
            self.launch_hook()

    def settle(self):
        if self.settle_hook is not None:
            self.settle_hook()

    # ---- plumbing ------------------------------------------------------------------
    def buffer(self, which) -> Tuple[int, int]:
        o, b = ctypes.c_uint64(), ctypes.c_uint64()
        C.check(self.L.dqnx_engine_buffer(self.h, which, ctypes.byref(o), ctypes.byref(b)), "buffer")
        return int(o.value), int(b.value)

    def view(self, which, dtype):
        o, b = self.buffer(which)
        t = self.arena[o:o + b]
        return t.view(dtype) if b else t.view(dtype)

    def stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def __del__(self):
        try:
            if getattr(self, "h", None):
                self.L.dqnx_engine_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def reset(self):
        C.check(self.L.dqnx_engine_reset(self.h, self.stream()), "reset")
        self.ring_size = 0
        self.ring_wptr = 0
        self.agent_step = 0

    def param_views(self, flat: torch.Tensor):
        """name -> view into a flat parameter vector, in state_dict order."""
        return {name: flat[off:off + int(np.prod(shape))].view(*shape) for name, off, shape in self.param_layout}

    def load_params(self, state: dict, target: Optional[dict] = None):
        for name, v in self.param_views(self.params).items():
            v.copy_(state[name].to(self.device, torch.float32))
        tsrc = state if target is None else target
        for name, v in self.param_views(self.target_params).items():
            v.copy_(tsrc[name].to(self.device, torch.float32))
        self.params_modified()

    def params_modified(self):
        """Call after writing `params` / `target_params` (or their state_dict views) directly:
        the next learn step rebuilds the engine's derived weight layouts (dqnx_params_modified).
        Adam, soft / hard updates and load_params keep them current by themselves."""
        C.check(self.L.dqnx_params_modified(self.h), "params_modified")

    # ---- replay ----------------------------------------------------------------------
    STAGE_ROWS = 64   # the library's pinned one-copy push block (dqnx_replay_push, <= 64 host rows)

    def push_host(self, obs, act, rew, done, next_obs, n: int):
        """The env loop's push (Agent.store_transitions, n_env rows of host data: numpy arrays or lists):
        the rows are written into preallocated host staging arrays whose addresses are cached, and one
        dqnx_replay_push call copies them on (one pinned block, one async copy).  numpy's per-array
        conversions and `.ctypes` lookups cost ~20 us per call on the old path; larger pushes take it."""
        if n > self.STAGE_ROWS:
            self.push(np.asarray(obs, dtype=np.float32).reshape(n, -1), np.asarray(act).reshape(n),
                      np.asarray(rew, dtype=np.float32).reshape(n), np.asarray(done).reshape(n),
                      np.asarray(next_obs, dtype=np.float32).reshape(n, -1))
            return
        st = getattr(self, "_stage", None)
        if st is None:
            D, R = self.spec.obs_dim, self.STAGE_ROWS
            arrs = (np.zeros((R, D), np.float32), np.zeros(R, np.int32), np.zeros(R, np.float32), np.zeros(R, np.uint8),
                    np.zeros((R, D), np.float32))
            st = self._stage = (arrs, tuple(a.__array_interface__["data"][0] for a in arrs))
        (o, a, r, d, no), (po, pa, pr, pd, pn) = st
        o[:n] = np.asarray(obs).reshape(n, -1)
        no[:n] = np.asarray(next_obs).reshape(n, -1)
        a[:n] = act
        r[:n] = rew
        d[:n] = done
        C.check(self.L.dqnx_replay_push(self.h, po, pa, pr, pd, pn, n, 0, self.stream()), "replay_push")
        self.ring_wptr = (self.ring_wptr + n) % self.capacity
        self.ring_size = min(self.ring_size + n, self.capacity)

    def push(self, obs, act, rew, done, next_obs):
        """Append transitions (numpy arrays or CUDA tensors)."""
        if isinstance(obs, torch.Tensor) and obs.is_cuda:
            obs = obs.contiguous().float()
            next_obs = next_obs.contiguous().float()
            act = act.to(torch.int32).contiguous()
            rew = rew.float().contiguous()
            done = done.to(torch.uint8).contiguous()
            n = obs.shape[0]
            C.check(self.L.dqnx_replay_push(self.h, obs.data_ptr(), act.data_ptr(), rew.data_ptr(), done.data_ptr(),
                                            next_obs.data_ptr(), n, 1, self.stream()), "replay_push")
        else:
            obs = np.ascontiguousarray(obs, dtype=np.float32).reshape(-1, self.spec.obs_dim)
            next_obs = np.ascontiguousarray(next_obs, dtype=np.float32).reshape(-1, self.spec.obs_dim)
            n = obs.shape[0]
            act = np.ascontiguousarray(act, dtype=np.int32).reshape(-1)
            rew = np.ascontiguousarray(rew, dtype=np.float32).reshape(-1)
            done = np.ascontiguousarray(np.asarray(done).astype(bool), dtype=np.uint8).reshape(-1)
            # (up to 64 rows -- the env loop's n_env -- the library packs them into its pinned block and
            # sends one async copy; larger pushes copy array by array and wait for the stream)
            C.check(self.L.dqnx_replay_push(self.h, obs.ctypes.data, act.ctypes.data, rew.ctypes.data,
                                            done.ctypes.data, next_obs.ctypes.data, n, 0, self.stream()),
                    "replay_push")
        self.ring_wptr = (self.ring_wptr + n) % self.capacity
        self.ring_size = min(self.ring_size + n, self.capacity)

    # ---- RNG -------------------------------------------------------------------------
    def set_rng(self, which: int, state625: np.ndarray):
        a = np.ascontiguousarray(state625, dtype=np.uint32)
        assert a.shape == (625,)
        C.check(self.L.dqnx_rng_set(self.h, which, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                    self.stream()), "rng_set")

    def get_rng(self, which: int) -> np.ndarray:
        a = np.empty(625, dtype=np.uint32)
        C.check(self.L.dqnx_rng_get(self.h, which, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                    self.stream()), "rng_get")
        return a

    # ---- the drop-in Agent's fast path (dqnx_agent_*: one library call per agent method) ----------
    def agent_stage_rng(self, which: int, state625) -> int:
        """Snapshot the caller's global RNG state for the next agent_launch; returns the MT19937 words
        the device draw will consume (the caller advances its generator by them).  state625: any buffer
        of 625 uint32 (an array.array('I') or a numpy array)."""
        if isinstance(state625, np.ndarray):
            ptr = state625.ctypes.data
        else:
            ptr = state625.buffer_info()[0]
        w = C.I64()
        C.check(self.L.dqnx_agent_stage_rng(self.h, which, ctypes.c_void_p(ptr), ctypes.byref(w)), "agent_stage_rng")
        return int(w.value)

    def agent_launch(self, soft_update: bool = False) -> None:
        C.check(self.L.dqnx_agent_launch(self.h, C.STEP_SOFT_UPDATE if soft_update else 0, self.stream()),
                "agent_launch")
        self._ag_unread = True
        if self.cfg.algo == C.DQNX_ALGO_PER_DOUBLE:   # every PER learn step samples: step += n_env
            self.agent_step += self.cfg.n_env

    def agent_learn_mt(self, mt_addr: int, pos_addr: int, launch: bool, soft_update: bool = False) -> int:
        """dqnx_agent_learn_mt (uniform replay): stage the live MT19937 at mt_addr / pos_addr for the
        device draw, advance it in place past the words the draw consumes, and (launch) launch the step
        as agent_launch does.  Returns the words consumed."""
        w = C.I64()
        flags = (C.AGENT_LAUNCH if launch else 0) | (C.STEP_SOFT_UPDATE if soft_update else 0)
        if launch and self._ag_unread:
            # the previous step's control block is still unread: wait for it here, through the CDLL
            # binding (GIL released), not inside dqnx_agent_learn_mt (GIL held for random._inst)
            C.check(self.L.dqnx_agent_quiesce(self.h), "agent_quiesce")
        C.check(self.L.dqnx_agent_learn_mt(self.h, mt_addr, pos_addr, flags, self.stream(), ctypes.byref(w)),
                "agent_learn_mt")
        self._ag_unread = self._ag_unread or launch
        return int(w.value)

    def agent_readback(self, wait: bool):
        """The control block of the last agent_launch once it has arrived (None: none pending / not
        yet); raises its sticky device error, or a mismatch between the device sampler's RNG state and
        the host mirror of the draw."""
        out = getattr(self, "_ag_ctrl", None)
        if out is None:
            out = self._ag_ctrl = C.Ctrl()
        rc = self.L.dqnx_agent_readback(self.h, 1 if wait else 0, ctypes.byref(out))
        if rc == 0:
            if wait:   # (nothing pending)
                self._ag_unread = False
            return None
        self._ag_unread = False
        if rc == C.DQNX_EDEVICE:
            if out.error:
                raise_device_error(out.error)
            raise RuntimeError("libdqnx: " + self.L.dqnx_last_error().decode(errors="replace"))
        C.check(rc if rc < 0 else 0, "agent_readback")
        return out

    # host-side RNG mirror (dqnx_rng_sample_words / dqnx_rng_advance; host only)
    def sample_words(self, state625: np.ndarray, n: int, k: int):
        """(words, state after) of CPython's random.sample(population of n, k) from `state625`."""
        out = np.empty(625, dtype=np.uint32)
        w = C.I64()
        C.check(self.L.dqnx_rng_sample_words(state625.ctypes.data, int(n), int(k), out.ctypes.data, ctypes.byref(w)),
                "rng_sample_words")
        return int(w.value), out

    def rng_advance(self, state625: np.ndarray, words: int) -> np.ndarray:
        out = np.empty(625, dtype=np.uint32)
        C.check(self.L.dqnx_rng_advance(state625.ctypes.data, int(words), out.ctypes.data), "rng_advance")
        return out

    # ---- steps -----------------------------------------------------------------------
    def set_graphs(self, on: bool):
        """Replay each learn step as a captured HIP graph (default) or launch its kernels one by
        one (e.g. into a caller's own stream capture)."""
        C.check(self.L.dqnx_engine_set_graphs(self.h, 1 if on else 0), "set_graphs")

    def learn_step(self, soft_update=False, given_indices=False, grads_only=False, prefetch=False):
        """One learn step (+ fused soft update).  prefetch=True also draws the next step's
        minibatch on a forked graph branch (pure learning loops; see DQNX_STEP_PREFETCH)."""
        flags = (C.STEP_SOFT_UPDATE if soft_update else 0) | (C.STEP_GIVEN_INDICES if given_indices else 0) \
            | (C.STEP_GRADS_ONLY if grads_only else 0) | (C.STEP_PREFETCH if prefetch else 0)
        C.check(self.L.dqnx_learn_step(self.h, flags, self.stream()), "learn_step")
        if self.cfg.algo == C.DQNX_ALGO_PER_DOUBLE:   # every PER learn step samples: step += n_env
            self.agent_step += self.cfg.n_env

    def prefetch_prologue(self, grads_only=True):
        """Draw the first minibatch of a prefetching loop now (dqnx_prefetch_begin)."""
        C.check(self.L.dqnx_prefetch_begin(self.h, C.STEP_GRADS_ONLY if grads_only else 0, self.stream()),
                "prefetch_begin")

    def learn_steps(self, count: int, soft_update=False):
        """`count` consecutive learn steps in one call (dqnx_learn_steps): bitwise equal to
        `count` learn_step(soft_update) calls; one graph on the fused MLP plan, with every step's
        minibatch after the first drawn inside the previous step's last launch."""
        C.check(self.L.dqnx_learn_steps(self.h, C.STEP_SOFT_UPDATE if soft_update else 0, int(count),
                                        self.stream()), "learn_steps")
        if self.cfg.algo == C.DQNX_ALGO_PER_DOUBLE:
            self.agent_step += self.cfg.n_env * int(count)

    def apply_grads(self, soft_update=False):
        C.check(self.L.dqnx_apply_grads(self.h, C.STEP_SOFT_UPDATE if soft_update else 0, self.stream()),
                "apply_grads")

    # ---- bucketed data-parallel step (dqn.data_parallel.dp_learn_step_bucketed) ----
    def dp_buckets(self):
        """[(first, count)] flat ranges of `grads` / `params`, in the order the backward completes
        them: dense layers + head (+ the loss slot) first, then the convs, last conv first."""
        n = ctypes.c_int32()
        C.check(self.L.dqnx_dp_bucket_count(self.h, ctypes.byref(n)), "dp_bucket_count")
        out = []
        for b in range(n.value):
            f, c = ctypes.c_int64(), ctypes.c_int64()
            C.check(self.L.dqnx_dp_bucket_info(self.h, b, ctypes.byref(f), ctypes.byref(c)), "dp_bucket_info")
            out.append((f.value, c.value))
        return out

    def learn_step_bucket(self, bucket: int, prefetch: bool = False):
        """The part of a GRADS_ONLY learn step that completes `bucket`'s gradient.  prefetch (fused MLP
        plan, bucket 0): the forward launch also draws the next step's minibatch (DQNX_STEP_PREFETCH)."""
        C.check(self.L.dqnx_learn_step_bucket(self.h, C.STEP_PREFETCH if prefetch else 0, int(bucket), self.stream()),
                "learn_step_bucket")
        if bucket == 0 and self.cfg.algo == C.DQNX_ALGO_PER_DOUBLE:   # bucket 0 samples: step += n_env
            self.agent_step += self.cfg.n_env

    def apply_grads_bucket(self, bucket: int, soft_update=False):
        """Adam (+ soft update) of `bucket`'s parameters from `grads` (bucket 0: + the PER tree update)."""
        C.check(self.L.dqnx_apply_grads_bucket(self.h, C.STEP_SOFT_UPDATE if soft_update else 0, int(bucket),
                                               self.stream()), "apply_grads_bucket")

    def soft_update(self):
        C.check(self.L.dqnx_soft_update(self.h, self.stream()), "soft_update")

    def hard_update(self):
        C.check(self.L.dqnx_hard_update(self.h, self.stream()), "hard_update")

    # ---- prioritised replay ------------------------------------------------------------
    def per_sample(self):
        """ReplayMemoryPrioritized.sample_transitions: slots -> batch_idx, IS weights -> is_weights."""
        C.check(self.L.dqnx_per_sample(self.h, self.stream()), "per_sample")
        self.agent_step += self.cfg.n_env

    def per_update_priorities(self, slots: torch.Tensor, abs_td: torch.Tensor):
        """update_batch_priorities(tree_indices, abs_td_errors) for device int32 ring slots
        and float32 |delta|, in order."""
        slots = slots.to(self.device, torch.int32).contiguous()
        abs_td = abs_td.to(self.device, torch.float32).contiguous()
        C.check(self.L.dqnx_per_update_priorities(self.h, ctypes.c_void_p(slots.data_ptr()),
                                                  ctypes.c_void_p(abs_td.data_ptr()), int(slots.numel()),
                                                  self.stream()), "per_update_priorities")

    # numpy's global legacy RandomState <-> the engine (PER draws np.random.uniform words)
    def set_np_state_from_global(self):
        st = np.random.get_state()
        self.set_rng(C.DQNX_RNG_NP, np.append(np.asarray(st[1], dtype=np.uint32), np.uint32(st[2])))

    def get_np_state_to_global(self):
        a = self.get_rng(C.DQNX_RNG_NP)
        st = np.random.get_state()
        np.random.set_state((st[0], a[:624].copy(), int(a[624]), st[3], st[4]))

    # CPython's global random state <-> the engine (the uniform sampler's random.sample)
    def set_py_state_from_global(self):
        self.set_rng(C.DQNX_RNG_PY, np.asarray(random.getstate()[1], dtype=np.uint32))

    def get_py_state_to_global(self):
        a = self.get_rng(C.DQNX_RNG_PY)
        v, _, g = random.getstate()
        random.setstate((v, tuple(int(x) for x in a), g))

    def set_agent_step(self, step_times_n_env: int):
        C.check(self.L.dqnx_set_agent_step(self.h, int(step_times_n_env), self.stream()), "set_agent_step")
        self.agent_step = int(step_times_n_env)

    def ctrl(self) -> C.Ctrl:
        """Snapshot of the device control block (synchronises)."""
        self.launch_recorded()
        raw = self.ctrl_bytes.cpu().numpy().tobytes()
        return C.Ctrl.from_buffer_copy(raw[:ctypes.sizeof(C.Ctrl)])

    def loss(self) -> float:
        return float(self.ctrl().loss)

    def check_device_error(self):
        raise_device_error(self.ctrl().error)


def raise_device_error(err: int):
    """The exception of a sticky dqnx_ctrl.error code (0: none)."""
    if err == C.DEVERR_SAMPLE_TOO_LARGE:
        raise ValueError("Sample larger than population or is negative")
    if err == C.DEVERR_EMPTY_TREE:
        raise RuntimeError("libdqnx: PER sample from a SumTree with total priority 0")
    if err == C.DEVERR_PER_HANDOFF:
        raise RuntimeError("libdqnx: PER tree update hand-off timed out inside a launch (internal error)")
    if err == C.DEVERR_FWD_PAIR_HANDOFF:
        raise RuntimeError("libdqnx: paired-column forward hand-off timed out inside a launch (internal error)")
    if err in C.DEVERR_BOUNDS:
        raise RuntimeError(f"libdqnx: out-of-range write skipped (internal error): {C.DEVERR_BOUNDS[err]}")
    if err:
        raise RuntimeError(f"libdqnx device error {err}")
