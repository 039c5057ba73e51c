"""oracle/ref.py -- TEST INFRASTRUCTURE ONLY (checker / CPU baseline, never the product).

torch-CPU + numpy restatement of the DQN learn-step path of
youcefMehamlia/Multimodal-DRL-RMC.  Every function cites the reference file:line it
restates (``R:`` = /root/reference/).  The reference itself is never imported here:
this module must run on the GPU box, where /root/reference does not exist.

Restated:
  * networks: MLP body (R:env/custom_env/macro with lane/dqn_config.py:58-104),
    TwoStreamHybridNetwork (R:env/dqn_config.py:66-143, network_config :148-193),
    DeepQNetwork / DuelingDeepQNetwork heads (R:dqn/network.py:50-117);
  * learn steps: SimpleAgent.learn (R:dqn/agent.py:166-185), DoubleAgent.learn
    (:204-226), PerDoubleAgent.learn (:245-272), transitions_to_tensor (:71-78);
  * torch.optim.Adam single-tensor path (torch 2.10 optim/adam.py
    _single_tensor_adam, the CPU default) and the soft/hard target update
    (R:dqn/agent.py:101-110);
  * replay: ReplayMemoryNaive (R:dqn/replay_memory.py:24-39) over a deque with
    CPython random.sample (restated in pyrandom.c), ReplayMemoryPrioritized
    (:43-98) and SumTree (R:dqn/utils/sum_tree.py:4-73) with numpy>=2 float64
    semantics.
"""
from __future__ import annotations

import ctypes
import math
import os
import random
from collections import OrderedDict, deque
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    """Load (building if needed) oracle/_build/liboracle.so."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = os.path.join(_HERE, "_build", "liboracle.so")
    if not os.path.exists(path):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", _HERE])
    L = ctypes.CDLL(path)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    L.oracle_genrand_uint32.argtypes = [u32p]
    L.oracle_genrand_uint32.restype = ctypes.c_uint32
    L.oracle_sample_setsize.argtypes = [ctypes.c_int64]
    L.oracle_sample_setsize.restype = ctypes.c_int64
    L.oracle_random_sample.argtypes = [u32p, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    L.oracle_random_sample.restype = ctypes.c_int
    L.oracle_np_random_sample.argtypes = [u32p]
    L.oracle_np_random_sample.restype = ctypes.c_double
    L.oracle_np_uniform.argtypes = [u32p, ctypes.c_double, ctypes.c_double]
    L.oracle_np_uniform.restype = ctypes.c_double
    _LIB = L
    return L


# ----------------------------------------------------------------------------------------
# RNG state helpers (Python random.getstate() / numpy get_state() <-> uint32[625])
# ----------------------------------------------------------------------------------------

def py_state_to_array(state=None) -> np.ndarray:
    """random.getstate() -> uint32[625] (624 MT words + index)."""
    st = random.getstate() if state is None else state
    return np.array(st[1], dtype=np.uint32)


def array_to_py_state(arr: np.ndarray, gauss_next=None):
    return (3, tuple(int(x) for x in arr.tolist()), gauss_next)


def np_state_to_array(state=None) -> np.ndarray:
    st = np.random.get_state() if state is None else state
    out = np.empty(625, dtype=np.uint32)
    out[:624] = st[1]
    out[624] = st[2]
    return out


def array_to_np_state(arr: np.ndarray, template=None):
    t = np.random.get_state() if template is None else template
    return ("MT19937", np.array(arr[:624], dtype=np.uint32), int(arr[624]), t[3], t[4])


def _u32p(a: np.ndarray):
    assert a.dtype == np.uint32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


def sample_positions(mt_state: np.ndarray, n: int, k: int) -> np.ndarray:
    """random.sample(population_of_len_n, k) as positions (R:dqn/replay_memory.py:39).
    Advances ``mt_state`` (uint32[625]) in place exactly like CPython."""
    out = np.empty(k, dtype=np.int64)
    rc = lib().oracle_random_sample(_u32p(mt_state), n, k,
                                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
    if rc != 0:
        raise ValueError("Sample larger than population or is negative")
    return out


def sample_setsize(k: int) -> int:
    return int(lib().oracle_sample_setsize(k))


def np_uniform(mt_state: np.ndarray, low: float, high: float) -> float:
    """numpy legacy RandomState.uniform(low, high) (R:dqn/replay_memory.py:80)."""
    return float(lib().oracle_np_uniform(_u32p(mt_state), low, high))


# ----------------------------------------------------------------------------------------
# Network specs and parameter init (module construction order = reference's)
# ----------------------------------------------------------------------------------------

@dataclass
class NetSpec:
    kind: str = "mlp"                  # "mlp" | "hybrid"
    obs_dim: int = 284
    n_actions: int = 8
    head: str = "dueling"              # "dueling" | "linear"
    hidden: Tuple[int, ...] = (256, 128)   # MLP body widths (R:.../macro with lane/dqn_config.py:75)
    # TwoStreamHybridNetwork (R:env/dqn_config.py:148-193)
    macro_len: int = 14
    micro_chw: Tuple[int, int, int] = (2, 27, 5)
    conv: Tuple[Tuple[int, Tuple[int, int], Tuple[int, int]], ...] = (
        (32, (3, 3), (1, 1)), (64, (3, 3), (2, 1)), (64, (3, 3), (2, 2)))
    dense: Tuple[int, ...] = (512, 256)

    @property
    def activation(self) -> str:
        return "relu" if self.kind == "mlp" else "elu"


def mlp_spec(obs_dim=284, n_actions=8, head="dueling", hidden=(256, 128)) -> NetSpec:
    return NetSpec(kind="mlp", obs_dim=obs_dim, n_actions=n_actions, head=head, hidden=tuple(hidden))


def hybrid_spec(n_actions=8, head="dueling", micro_chw=(2, 27, 5), macro_len=14) -> NetSpec:
    c, h, w = micro_chw
    return NetSpec(kind="hybrid", obs_dim=macro_len + c * h * w, n_actions=n_actions, head=head,
                   macro_len=macro_len, micro_chw=tuple(micro_chw))


def conv_out_hw(spec: NetSpec):
    c, h, w = spec.micro_chw
    dims = []
    for f, (kh, kw), (sh, sw) in spec.conv:
        ph, pw = kh // 2, kw // 2
        h = (h + 2 * ph - kh) // sh + 1
        w = (w + 2 * pw - kw) // sw + 1
        dims.append((f, h, w))
    return dims


def _build_modules(spec: NetSpec) -> "OrderedDict[str, nn.Module]":
    """Construct the torch layers in the reference's order; names = state_dict prefixes."""
    mods: "OrderedDict[str, nn.Module]" = OrderedDict()
    if spec.kind == "mlp":
        d = spec.obs_dim
        for i, hdim in enumerate(spec.hidden):        # nn.Sequential(Linear, act, Linear, act)
            mods[f"net.{2 * i}"] = nn.Linear(d, hdim)
            d = hdim
        fout = d
    else:
        c = spec.micro_chw[0]
        for i, (f, k, s) in enumerate(spec.conv):     # R:env/dqn_config.py:92-101
            mods[f"net.cnn_stream.{2 * i}"] = nn.Conv2d(c, f, kernel_size=k, stride=s,
                                                        padding=(k[0] // 2, k[1] // 2))
            c = f
        f, h, w = conv_out_hw(spec)[-1]
        d = f * h * w + spec.macro_len                  # R:env/dqn_config.py:104-113
        for i, o in enumerate(spec.dense):              # R:env/dqn_config.py:116-122
            mods[f"net.dense_stream.{2 * i}"] = nn.Linear(d, o)
            d = o
        fout = d
    if spec.head == "dueling":                          # R:dqn/network.py:81-82
        mods["fc_val"] = nn.Linear(fout, 1)
        mods["fc_adv"] = nn.Linear(fout, spec.n_actions)
    else:                                               # R:dqn/network.py:54
        mods["fc_out"] = nn.Linear(fout, spec.n_actions)
    return mods


def _params_of(mods) -> "OrderedDict[str, torch.Tensor]":
    out = OrderedDict()
    for name, m in mods.items():
        out[name + ".weight"] = m.weight.detach().clone()
        out[name + ".bias"] = m.bias.detach().clone()
    return out


def reference_init(spec: NetSpec, seed: int) -> "OrderedDict[str, torch.Tensor]":
    """Initial online parameters as the reference agent constructor produces them after
    ``torch.manual_seed(seed)``: online net built, then target net built (consuming the
    RNG), then target <- online (R:dqn/agent.py:299-308, :101-103)."""
    torch.manual_seed(seed)
    online = _params_of(_build_modules(spec))
    _build_modules(spec)  # target net construction consumes the same RNG stream
    return online


def param_count(spec: NetSpec) -> int:
    return sum(p.numel() for p in reference_init(spec, 0).values())


# ----------------------------------------------------------------------------------------
# Forward (functional restatement of the module forwards)
# ----------------------------------------------------------------------------------------

def bf16r(t: torch.Tensor) -> torch.Tensor:
    """Round to bf16 (round to nearest even) and back to fp32."""
    return t.to(torch.bfloat16).to(torch.float32)


class _Bf16Linear(torch.autograd.Function):
    """The engine's bf16 compute mode (include/dqnx.h DQNX_COMPUTE_BF16), restated: GEMM
    operands rounded to bf16, products summed in fp32.  Not in the reference (fp32 only);
    this is the checker for BASELINE config 5's bf16 variant.
      y  = bf16(x) bf16(W)^T + b
      dx = bf16(dy) bf16(W)   (dense layers >= 2: the engine's dZ chain)  /  dy W  (head)
      dW = bf16(dy)^T bf16(x), db = sum bf16(dy)   (k_dw_bf16: the bias is the ones column)"""

    @staticmethod
    def forward(ctx, x, W, b, round_dx):
        ctx.save_for_backward(x, W)
        ctx.round_dx = round_dx
        return bf16r(x) @ bf16r(W).t() + b

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        dx = bf16r(dy) @ bf16r(W) if ctx.round_dx else dy @ W
        dyr = bf16r(dy)
        return dx, dyr.t() @ bf16r(x), dyr.sum(0), None


def _linear(x, W, b, bf16: bool, round_dx: bool = True):
    return _Bf16Linear.apply(x, W, b, round_dx) if bf16 else F.linear(x, W, b)


def body_forward(spec: NetSpec, P, x: torch.Tensor, bf16: bool = False) -> torch.Tensor:
    if spec.kind == "mlp":   # R:env/custom_env/macro with lane/dqn_config.py:76-84
        h = x
        for i in range(len(spec.hidden)):
            h = torch.relu(_linear(h, P[f"net.{2 * i}.weight"], P[f"net.{2 * i}.bias"], bf16))
        return h
    assert not bf16, "bf16 compute is implemented for MLP networks only"
    # TwoStreamHybridNetwork.forward (R:env/dqn_config.py:118-143)
    L = spec.macro_len
    macro = x[:, :L]
    micro = x[:, L:].view(-1, *spec.micro_chw)
    h = micro
    for i, (f, k, s) in enumerate(spec.conv):
        h = F.elu(F.conv2d(h, P[f"net.cnn_stream.{2 * i}.weight"], P[f"net.cnn_stream.{2 * i}.bias"],
                           stride=s, padding=(k[0] // 2, k[1] // 2)))
    h = torch.cat([h.flatten(start_dim=1), macro], dim=1)
    for i in range(len(spec.dense)):
        h = F.elu(F.linear(h, P[f"net.dense_stream.{2 * i}.weight"], P[f"net.dense_stream.{2 * i}.bias"]))
    return h


def q_forward(spec: NetSpec, P, x: torch.Tensor, bf16: bool = False) -> torch.Tensor:
    h = body_forward(spec, P, x, bf16)
    if spec.head == "dueling":   # R:dqn/network.py:90-96 (aggregate :83)
        val = _linear(h, P["fc_val.weight"], P["fc_val.bias"], bf16, round_dx=False)
        adv = _linear(h, P["fc_adv.weight"], P["fc_adv.bias"], bf16, round_dx=False)
        return torch.add(val, (adv - adv.mean(dim=1, keepdim=True)))
    return _linear(h, P["fc_out.weight"], P["fc_out.bias"], bf16, round_dx=False)   # R:dqn/network.py:61-65


def advantages(spec: NetSpec, P, x: torch.Tensor) -> torch.Tensor:
    h = body_forward(spec, P, x)
    return F.linear(h, P["fc_adv.weight"], P["fc_adv.bias"])


def greedy_actions(spec: NetSpec, P, obs: np.ndarray) -> List[int]:
    """Network.actions (R:dqn/network.py:67-74; dueling uses advantages, :110-117)."""
    x = torch.as_tensor(obs, dtype=torch.float32)
    with torch.no_grad():
        q = advantages(spec, P, x) if spec.head == "dueling" else q_forward(spec, P, x)
    return torch.argmax(q, dim=1).tolist()


# ----------------------------------------------------------------------------------------
# Replay memories
# ----------------------------------------------------------------------------------------

class NaiveReplay:
    """ReplayMemoryNaive (R:dqn/replay_memory.py:24-39): deque + random.sample."""

    def __init__(self, buffer_size: int, batch_size: int):
        self.batch_size = batch_size
        self.buffer_size = buffer_size
        self.replay_buffer = deque(maxlen=buffer_size)

    def store_transitions(self, obses, actions, rews, dones, new_obses):
        for e, (obs, action, rew, done, new_obs) in enumerate(zip(obses, actions, rews, dones, new_obses)):
            self.replay_buffer.append((obs, action, rew, done, new_obs))
            if done:
                yield e

    def sample_positions(self, mt_state: np.ndarray) -> np.ndarray:
        return sample_positions(mt_state, len(self.replay_buffer), self.batch_size)

    def sample_transitions(self, mt_state: np.ndarray):
        pos = self.sample_positions(mt_state)
        buf = self.replay_buffer
        return [buf[int(j)] for j in pos], pos


class SumTree:
    """SumTree (R:dqn/utils/sum_tree.py:4-73), numpy>=2 float64 semantics by default.

    numpy121=True restates the reference's pinned numpy 1.21 (R:bin/environment.yml) for the
    float32 (1,)-array priorities update_batch_priorities passes (R:dqn/replay_memory.py:95-98):
    value-based casting casts the float64 tree scalar down, so `change = priority - tree[i]`
    (:18) and `tree[parent] += change` (:31-32) are float32 operations whose results are stored
    back into the float64 tree.  Pushes (float64 scalar priorities, :34-40) stay float64 under
    both versions.  numpy 1.21 is not installed here: this mode is a restatement of the casting
    rules (parity unpinned against a numpy 1.21 run)."""

    def __init__(self, capacity: int, numpy121: bool = False):
        self.numpy121 = numpy121
        self.capacity = capacity
        self.tree = np.zeros(2 * capacity - 1)
        self.data = [None] * capacity
        self.data_pointer = 0
        self.size = 0
        self.max_priority_index = capacity - 1
        self.min_priority_index = capacity - 1

    def update(self, tree_index: int, priority: float, f32: bool = False):   # :15-32
        tree = self.tree
        max_p, min_p = tree[self.max_priority_index], tree[self.min_priority_index]
        f32 = f32 and self.numpy121
        if f32:   # numpy 1.21: float32 array minus float64 scalar -> float32
            priority = float(np.float32(priority))
            change = np.float32(np.float32(priority) - np.float32(tree[tree_index]))
        else:
            priority = float(priority)
            change = priority - tree[tree_index]
        tree[tree_index] = priority
        lo, hi = self.capacity - 1, self.capacity + self.size - 1
        if priority >= max_p:
            self.max_priority_index = tree_index
        elif tree_index == self.max_priority_index:
            self.max_priority_index = int(np.argmax(tree[lo:hi])) + lo
        if priority <= min_p:
            self.min_priority_index = tree_index
        elif tree_index == self.min_priority_index:
            self.min_priority_index = int(np.argmin(tree[lo:hi])) + lo
        while tree_index != 0:
            tree_index = (tree_index - 1) // 2
            if f32:   # float64 scalar + float32 array -> float32, stored into the float64 tree
                tree[tree_index] = float(np.float32(np.float32(tree[tree_index]) + change))
            else:
                tree[tree_index] += change

    def add(self, priority: float, data):                      # :34-40
        tree_index = self.data_pointer + self.capacity - 1
        self.data[self.data_pointer] = data
        self.data_pointer = (self.data_pointer + 1) % self.capacity
        self.size = min(self.size + 1, self.capacity)
        self.update(tree_index, priority)

    def get_leaf(self, v: float):                              # :42-61
        tree = self.tree
        parent = 0
        n = len(tree)
        while True:
            left = 2 * parent + 1
            if left >= n:
                leaf = parent
                break
            if v <= tree[left]:
                parent = left
            else:
                v -= tree[left]
                parent = left + 1
        return leaf, tree[leaf], self.data[leaf - self.capacity + 1]

    @property
    def total_priority(self):
        return self.tree[0]

    @property
    def max_priority(self):
        return self.tree[self.max_priority_index]

    @property
    def min_priority(self):
        return self.tree[self.min_priority_index]


class PerReplay:
    """ReplayMemoryPrioritized (R:dqn/replay_memory.py:43-98)."""

    def __init__(self, buffer_size: int, batch_size: int, eps_dec: float, pow_mode: str = "numpy",
                 numpy121: bool = False):
        self.pow_mode = pow_mode
        self.batch_size = batch_size
        self.buffer_size = buffer_size
        self.replay_buffer = SumTree(buffer_size, numpy121=numpy121)
        self.epsilon = 0.0001
        self.alpha = 0.6
        self.beta_start = 0.4
        self.beta_end = 1.0
        self.beta_inc = eps_dec
        self.max_priority_high = 1.0

    def store_transitions(self, obses, actions, rews, dones, new_obses):   # :56-67
        max_priority = self.replay_buffer.max_priority
        if max_priority == 0:
            max_priority = self.max_priority_high
        for e, (obs, action, rew, done, new_obs) in enumerate(zip(obses, actions, rews, dones, new_obses)):
            self.replay_buffer.add(max_priority, (obs, action, rew, done, new_obs))
            if done:
                yield e

    def beta(self, step) -> float:
        return float(np.interp(step, [0, self.beta_inc], [self.beta_start, self.beta_end]))

    def sample_transitions(self, step, np_state: np.ndarray):          # :69-92
        t = self.replay_buffer
        seg = t.total_priority / self.batch_size
        beta = np.interp(step, [0, self.beta_inc], [self.beta_start, self.beta_end])
        prob_min = t.min_priority / t.total_priority
        max_w = np.power(np.float64(t.size * prob_min), -beta)
        is_w, idxs, trans = [], [], []
        for i in range(self.batch_size):
            v = np_uniform(np_state, float(seg * i), float(seg * (i + 1)))
            leaf, p, data = t.get_leaf(v)
            prob = p / t.total_priority
            w = np.power(np.float64(t.size * prob), -beta) / max_w
            is_w.append(float(w))
            idxs.append(leaf)
            trans.append(data)
        return is_w, idxs, trans

    def priorities(self, abs_td_errors_np: np.ndarray) -> np.ndarray:
        """float32 p = min(|d| + eps, 1)^alpha  (R:dqn/replay_memory.py:95).

        pow_mode "numpy": this host's numpy float32 power, which is what the reference computes
        when run here (numpy >= 1.22 on AVX-512 dispatches to SVML, within 1 ulp of correctly
        rounded).  pow_mode "cr": correctly rounded float32 power (float64 pow rounded once),
        which is glibc powf's result (the reference's pinned numpy 1.21 calls libm powf) except
        in rare hard cases; libdqnx computes this."""
        x = np.minimum(abs_td_errors_np + self.epsilon, self.max_priority_high)
        if self.pow_mode == "cr":
            return np.power(x.astype(np.float64), np.float64(np.float32(self.alpha))).astype(np.float32)
        return np.power(x, self.alpha)

    def update_batch_priorities(self, tree_indices, abs_td_errors_np):  # :94-98
        pr = self.priorities(abs_td_errors_np).reshape(-1)
        for i, p in zip(tree_indices, pr):   # float32 (1,) arrays in the reference
            self.replay_buffer.update(int(i), float(p), f32=True)


def transitions_to_tensor(transitions):
    """Agent.transitions_to_tensor (R:dqn/agent.py:71-78) on CPU."""
    obses_t = torch.as_tensor(np.asarray([t[0] for t in transitions]), dtype=torch.float32)
    actions_t = torch.as_tensor(np.asarray([t[1] for t in transitions]), dtype=torch.int64).unsqueeze(-1)
    rews_t = torch.as_tensor(np.asarray([t[2] for t in transitions]), dtype=torch.float32).unsqueeze(-1)
    dones_t = torch.as_tensor(np.asarray([t[3] for t in transitions]), dtype=torch.float32).unsqueeze(-1)
    new_obses_t = torch.as_tensor(np.asarray([t[4] for t in transitions]), dtype=torch.float32)
    return obses_t, actions_t, rews_t, dones_t, new_obses_t


# ----------------------------------------------------------------------------------------
# Optimizer / target update
# ----------------------------------------------------------------------------------------

def adam_update(p, g, m, v, step: int, lr: float, betas=(0.9, 0.999), eps=1e-8):
    """torch.optim.Adam single-tensor step (torch 2.10 optim/adam.py _single_tensor_adam,
    non-capturable branch), amsgrad=False, weight_decay=0, maximize=False."""
    beta1, beta2 = betas
    m.lerp_(g, 1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bias_correction1 = 1 - beta1 ** step
    bias_correction2 = 1 - beta2 ** step
    step_size = lr / bias_correction1
    bias_correction2_sqrt = bias_correction2 ** 0.5
    denom = (v.sqrt() / bias_correction2_sqrt).add_(eps)
    p.addcdiv_(m, denom, value=-step_size)


def soft_update(target, online, tau: float, n_env: int):
    """R:dqn/agent.py:105-110."""
    for k in target:
        target[k].copy_((tau * n_env) * online[k] + (1. - (tau * n_env)) * target[k])


# ----------------------------------------------------------------------------------------
# Learner (Agent.learn restatements)
# ----------------------------------------------------------------------------------------

ALGOS = ("DQNAgent", "DoubleDQNAgent", "DuelingDoubleDQNAgent", "PerDuelingDoubleDQNAgent")


def algo_spec_head(algo: str) -> str:
    return "dueling" if algo in ("DuelingDoubleDQNAgent", "PerDuelingDoubleDQNAgent") else "linear"


@dataclass
class StepRecord:
    positions: np.ndarray = None       # sampled logical replay positions (uniform) / tree leaves (PER)
    q_online_next: torch.Tensor = None
    q_target_next: torch.Tensor = None
    q_online: torch.Tensor = None
    targets: torch.Tensor = None
    loss: float = 0.0
    grads: "OrderedDict[str, torch.Tensor]" = None
    is_weights: Optional[np.ndarray] = None
    abs_td: Optional[np.ndarray] = None


class OracleLearner:
    """One agent's learn-step state: online/target params, Adam moments, replay, RNG states.

    ``learn()`` + ``update_target_network()`` is exactly the unit train.py executes per
    step (R:train.py:99-101)."""

    def __init__(self, spec: NetSpec, algo: str, batch_size: int, buffer_size: int,
                 lr=1e-4, gamma=0.99, tau=1e-3, n_env=1, soft_update=True,
                 update_target_frequency=30000, eps_dec=2e6, seed=0, params=None, per_pow="numpy",
                 compute="fp32", per_numpy121=False):
        assert algo in ALGOS and compute in ("fp32", "bf16")
        self.bf16 = compute == "bf16"
        self.spec, self.algo = spec, algo
        self.batch_size, self.buffer_size = batch_size, buffer_size
        self.lr, self.gamma, self.tau, self.n_env = lr, gamma, tau, n_env
        self.target_soft_update = soft_update
        self.update_target_frequency = update_target_frequency
        self.online = reference_init(spec, seed) if params is None else \
            OrderedDict((k, v.detach().clone().float()) for k, v in params.items())
        self.target = OrderedDict((k, v.clone()) for k, v in self.online.items())
        self.m = OrderedDict((k, torch.zeros_like(v)) for k, v in self.online.items())
        self.v = OrderedDict((k, torch.zeros_like(v)) for k, v in self.online.items())
        self.adam_step = 0
        self.step = 0
        self.per = algo == "PerDuelingDoubleDQNAgent"
        self.replay = PerReplay(buffer_size, batch_size, eps_dec, per_pow, per_numpy121) if self.per \
            else NaiveReplay(buffer_size, batch_size)
        self.py_state = py_state_to_array(random.getstate())
        self.np_state = np_state_to_array(np.random.get_state())

    # -- store (R:dqn/agent.py:80-84)
    def store_transitions(self, obses, actions, rews, dones, new_obses):
        return list(self.replay.store_transitions(obses, actions, rews, dones, new_obses))

    def _q(self, P, x):
        return q_forward(self.spec, P, x, self.bf16)

    def learn(self, shard: Optional[Tuple[int, int]] = None) -> StepRecord:
        """Agent.learn.  With shard=(b0, b1) (data-parallel restatement) the loss
        is the shard's share of the global-batch mean, only the gradient is produced (no Adam,
        no priority update) and apply_grads() finishes the step with the all-reduced sum."""
        rec = StepRecord()
        B = self.batch_size
        if self.per:
            is_w, idxs, transitions = self.replay.sample_transitions(self.step * self.n_env, self.np_state)
            rec.positions = np.asarray(idxs, dtype=np.int64)
            rec.is_weights = np.asarray(is_w, dtype=np.float64)
            is_weights_t = torch.as_tensor(np.asarray(is_w), dtype=torch.float32).unsqueeze(-1)
        else:
            transitions, pos = self.replay.sample_transitions(self.py_state)
            rec.positions = pos
        obses_t, actions_t, rews_t, dones_t, new_obses_t = transitions_to_tensor(transitions)

        with torch.no_grad():
            if self.algo == "DQNAgent":                       # R:dqn/agent.py:171-175
                tq = self._q(self.target, new_obses_t)
                rec.q_target_next = tq
                sel = tq.max(dim=1, keepdim=True)[0]
            else:                                             # R:dqn/agent.py:209-214
                oq = self._q(self.online, new_obses_t)
                rec.q_online_next = oq
                best = oq.argmax(dim=1, keepdim=True)
                tq = self._q(self.target, new_obses_t)
                rec.q_target_next = tq
                sel = torch.gather(input=tq, dim=1, index=best)
            targets = rews_t + (1 - dones_t) * self.gamma * sel
        rec.targets = targets

        params = OrderedDict((k, v.detach().clone().requires_grad_(True)) for k, v in self.online.items())
        q = self._q(params, obses_t)
        rec.q_online = q.detach()
        qa = torch.gather(input=q, dim=1, index=actions_t)
        if self.per:                                          # R:dqn/agent.py:263-267
            with torch.no_grad():
                abs_td = torch.abs(targets - qa).detach().cpu().numpy()
                rec.abs_td = abs_td
                if shard is None:
                    self.replay.update_batch_priorities(rec.positions.tolist(), abs_td)
            per_sample = is_weights_t * F.smooth_l1_loss(qa, targets, reduction="none")
            loss = torch.mean(per_sample) if shard is None else per_sample[shard[0]:shard[1]].sum() / B
        elif shard is None:
            loss = F.smooth_l1_loss(qa, targets, reduction="mean")
        else:
            loss = F.smooth_l1_loss(qa[shard[0]:shard[1]], targets[shard[0]:shard[1]], reduction="sum") / B
        rec.loss = float(loss.item())
        grads = torch.autograd.grad(loss, list(params.values()))
        rec.grads = OrderedDict(zip(params.keys(), [g.detach() for g in grads]))
        if shard is None:
            self.apply_grads(rec.grads)
        return rec

    def apply_grads(self, grads, abs_td=None, positions=None):
        """optimizer.step() with the given (all-reduced) gradient; under DP also the PER
        priority update from the all-gathered |delta|."""
        if self.per and abs_td is not None:
            self.replay.update_batch_priorities(list(positions), np.asarray(abs_td, dtype=np.float32).reshape(-1, 1))
        self.adam_step += 1
        with torch.no_grad():
            for k in self.online:
                adam_update(self.online[k], grads[k], self.m[k], self.v[k], self.adam_step, self.lr)

    def update_target_network(self, force=False):             # R:dqn/agent.py:101-110
        if (not self.target_soft_update and self.step % (self.update_target_frequency // self.n_env) == 0) or force:
            for k in self.target:
                self.target[k].copy_(self.online[k])
        elif self.target_soft_update:
            with torch.no_grad():
                soft_update(self.target, self.online, self.tau, self.n_env)

    def train_step(self) -> StepRecord:
        """learn() then update_target_network(): the R:train.py:99-101 unit."""
        rec = self.learn()
        self.update_target_network()
        self.step += 1
        return rec


# ----------------------------------------------------------------------------------------
# Synthetic 1ramp_1x3 transitions
# ----------------------------------------------------------------------------------------

def synth_transitions(n: int, obs_dim: int = 284, n_actions: int = 8, seed: int = 0,
                      macro_len: int = 14):
    """numpy default_rng(seed) synthetic transitions shaped like the 1ramp_1x3 env:
    macro features U[0,1); micro grid HWC (27,5,2) occupancy ~ Bernoulli(0.2) with
    speed ~ U[0,1) where occupied (R:env/custom_env/sumo_env.py:296-301); action U{0..7};
    reward U[-24, 3] (R:env/custom_env/rl_controller.py:391-423); done ~ Bernoulli(1/90)."""
    rng = np.random.default_rng(seed)

    def obs_block():
        o = np.empty((n, obs_dim), dtype=np.float32)
        m = min(macro_len, obs_dim)
        o[:, :m] = rng.random((n, m), dtype=np.float32)
        g = obs_dim - m
        if g > 0:
            occ = rng.random((n, g), dtype=np.float32) < 0.2
            spd = rng.random((n, g), dtype=np.float32)
            o[:, m:] = np.where(occ, spd, np.float32(0.0))
        return o

    obs = obs_block()
    new_obs = obs_block()
    act = rng.integers(0, n_actions, size=n, dtype=np.int64)
    rew = (rng.random(n, dtype=np.float64) * 27.0 - 24.0).astype(np.float32)
    done = rng.random(n) < (1.0 / 90.0)
    return obs, act, rew, done, new_obs


def fill_replay(learner: OracleLearner, obs, act, rew, done, new_obs):
    """Push transitions one env-step at a time (n_env=1), like init_replay_memory_buffer
    (R:train.py:63-81)."""
    for i in range(len(act)):
        list(learner.replay.store_transitions(obs[i:i + 1], [int(act[i])], [float(rew[i])],
                                              [bool(done[i])], new_obs[i:i + 1]))
