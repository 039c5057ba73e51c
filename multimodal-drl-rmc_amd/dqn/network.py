"""Drop-in `dqn.network`: the reference's Q-network classes (R:dqn/network.py:11-117).

The classes keep the reference's constructor, attribute and method surface
(`Net(device, lr, nn_conf_func, input_dim, output_dim, reduction)`, `.net`, `.fc_out` /
`.fc_val` + `.fc_adv`, `.optimizer`, `.loss`, `forward`, `actions`, `value`, `advantages`,
`save`, `load`, `state_dict()` keys), so `Agents` / Observe code constructs them unchanged.

When an agent owns the network, `bind_flat()` re-points every parameter at its slice of
the learn engine's flat fp32 buffer (online or target).  From then on `state_dict()`,
`load_state_dict()`, `save()` and `forward()` read and write the same HBM the engine
trains, with no copies.  The engine (not `.optimizer`) holds the Adam moments; see
`dqn.agent`.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch as T
import torch.nn as nn

from . import _capi as C
from .engine import act as _act_native
from .engine import act_scratch, act_supported
from .engine import spec_from_body
from .utils.pack import load_pack, save_pack


class Network(nn.Module):
    """R:dqn/network.py:11-47."""

    def __init__(self, device, nn_conf_func, input_dim):
        super().__init__()
        self.net, self.fc_out_dim, optim_func, loss_func = nn_conf_func(input_dim)
        self.optim_func = (lambda params, lr: optim_func(params, lr=lr))
        self.loss_func = (lambda reduction: loss_func(reduction=reduction))
        self.device = device
        self._act_spec = None       # NetSpec of the acting kernel (None: not yet planned)
        self._act_flat = None       # flat fp32 parameter buffer the acting kernel reads
        self._act_params = None     # the Parameter objects bound to _act_flat
        self._act_ptrs = None       # their data_ptr when _act_flat was bound
        self._act_engine = False    # _act_flat belongs to a learn engine
        self._act_fast = None       # dqnx_act_host's arguments (scratch, staging, addresses), built once
        self._engine = None         # the learn engine whose buffer holds these parameters

    def forward(self, s):
        raise NotImplementedError

    def actions(self, obses):
        raise NotImplementedError

    def _engine_sync(self):
        """An agent's recorded learn step is launched before anything reads these parameters (stream
        order does the rest), so every read sees the post-step weights as after the reference's
        synchronous learn() (R:dqn/agent.py:204-226)."""
        eng = getattr(self, "_engine", None)
        if eng is not None:
            eng.launch_recorded()

    def named_parameters(self, *args, **kwargs):   # (parameters() goes through it)
        self._engine_sync()
        return super().named_parameters(*args, **kwargs)

    # -- engine binding -------------------------------------------------------------
    def bind_flat(self, views: dict, flat=None, spec=None, engine=None):
        """Move every parameter into `views[name]` (same shape, engine memory), keeping
        the Parameter objects (so `.optimizer` and module references stay valid).  With
        `flat`/`spec` (the learn engine's buffer and network description) `actions()` runs
        the acting kernel straight on that buffer."""
        with T.no_grad():
            for name, p in self.named_parameters():
                v = views[name]
                if tuple(v.shape) != tuple(p.shape):
                    raise ValueError(f"{name}: engine shape {tuple(v.shape)} != {tuple(p.shape)}")
                v.copy_(p.data.to(v.device, T.float32))
                p.data = v
        self._engine = engine
        if engine is not None:
            engine.params_modified()
        if flat is not None:
            self._act_flat, self._act_spec, self._act_engine = flat, spec, True
            self._act_remember_params()

    def _act_remember_params(self):
        """The Parameter objects and their storage addresses the acting kernels were bound to: each act
        checks the addresses against these objects (a few data_ptr() calls; walking the module tree
        through parameters() cost ~12 us per call)."""
        self._act_params = [p for _, p in super().named_parameters()]
        self._act_ptrs = [p.data_ptr() for p in self._act_params]
        self._act_fast = None

    # -- acting path: one dqnx_act launch for MLP bodies on a GPU -----------------------
    def _act_head_dim(self):
        head = self.fc_adv if hasattr(self, "fc_adv") else self.fc_out
        return head.out_features

    def _act_gpu(self, obses, na=None):
        """Greedy actions through the acting kernel: host obs -> dqnx_act_host (obs through pinned memory,
        one launch sequence, actions back, one synchronisation); device obs -> dqnx_act."""
        self._engine_sync()   # a recorded learn step first (stream order does the rest)
        spec, flat = na if na is not None else self._native_act()
        if isinstance(obses, T.Tensor) and obses.is_cuda:
            x = obses.reshape(obses.shape[0], -1)
            out = _act_native(spec, flat, x, scratch=act_scratch(spec, x.shape[0], flat.device))
            return out.cpu().tolist()
        x = obses if isinstance(obses, np.ndarray) else np.asarray(obses, dtype=np.float32)
        n = x.shape[0]
        f = self._act_fast
        if f is None or f[0] < n or f[1] is not spec or f[2] is not flat:
            L = C.lib()
            desc = spec.to_c()
            cap = max(n, 64)
            nb = int(L.dqnx_act_host_scratch_bytes(ctypes.byref(desc), cap))
            scratch = T.zeros((nb + 15) // 16 * 4, dtype=T.float32, device=flat.device)
            xs = np.zeros((cap, spec.obs_dim), dtype=np.float32)
            out = np.zeros(cap, dtype=np.int32)
            # (the acting launch's arguments, addresses resolved once)
            f = self._act_fast = (cap, spec, flat, desc, ctypes.byref(desc), flat.data_ptr(), scratch,
                                  scratch.data_ptr(), scratch.numel() * 4, xs, xs.__array_interface__["data"][0],
                                  out, out.__array_interface__["data"][0])
        _, _, _, _, dref, fptr, _, sptr, nbytes, xs, xaddr, out, oaddr = f
        xs[:n] = x.reshape(n, -1)
        stream = T.cuda.current_stream(flat.device).cuda_stream
        C.check(C.lib().dqnx_act_host(dref, fptr, xaddr, n, oaddr, sptr, nbytes, stream), "act_host")
        return out[:n].tolist()

    def _body_obs_dim(self):
        if isinstance(self.net, nn.Sequential):
            return self.net[0].in_features
        c, h, w = (int(x) for x in self.net.micro_shape)   # TwoStreamHybridNetwork
        return int(self.net.macro_len) + c * h * w

    def _native_act(self):
        """(spec, flat) for the acting kernels, or None when the reference's torch forward is
        the path: a CPU device (the caller asked for CPU) or a body outside the two families
        the engine implements."""
        if T.device(self.device).type != "cuda":
            return None
        if self._act_flat is not None:
            if not act_supported(self._act_spec):
                return None
            if all(p.data_ptr() == q for p, q in zip(self._act_params, self._act_ptrs)):
                return self._act_spec, self._act_flat
            if self._act_engine:
                raise RuntimeError("network parameters were moved out of the learn engine's buffer")
        # standalone network (e.g. Observe): pack its parameters into one flat buffer once.  A
        # body outside the two reference families keeps the reference's torch forward.
        try:
            spec = spec_from_body(self.net, self._body_obs_dim(), self._act_head_dim(),
                                  dueling=hasattr(self, "fc_adv"))
        except (NotImplementedError, AttributeError, TypeError, IndexError):
            return None
        if not act_supported(spec):
            return None
        n, layout = spec.param_infos()
        dev = next(self.parameters()).device
        flat = T.empty(n, dtype=T.float32, device=dev)
        views = {name: flat[off:off + int(T.Size(shape).numel())].view(*shape) for name, off, shape in layout}
        self.bind_flat(views)
        self._act_spec, self._act_flat, self._act_engine = spec, flat, False
        self._act_remember_params()
        return spec, flat

    # -- checkpoints (R:dqn/network.py:27-47; format: dqn.utils.pack) -----------------
    def save(self, save_path, step, episode_count, rew_mean, len_mean):
        params = {k: v.detach().cpu().numpy() for k, v in self.state_dict().items()}
        save_pack(save_path, params, step, episode_count, rew_mean, len_mean)

    def load(self, load_path):
        params, step, episode_count, rew_mean, len_mean = load_pack(load_path)
        self.load_state_dict({k: T.as_tensor(v, device=self.device) for k, v in params.items()})
        return step, episode_count, rew_mean, len_mean

    def state_dict(self, *args, **kwargs):
        self._engine_sync()
        return super().state_dict(*args, **kwargs)

    def load_state_dict(self, state_dict, *args, **kwargs):
        self._engine_sync()
        out = super().load_state_dict(state_dict, *args, **kwargs)
        if self._engine is not None:   # written into the engine's buffer: refresh its derived layouts
            self._engine.params_modified()
        return out


class DeepQNetwork(Network):
    """R:dqn/network.py:50-74."""

    def __init__(self, device, lr, nn_conf_func, input_dim, output_dim, reduction='mean'):
        super().__init__(device, nn_conf_func, input_dim)
        self.fc_out = nn.Linear(self.fc_out_dim, output_dim)
        self.optimizer = self.optim_func(self.parameters(), lr=lr)
        self.loss = self.loss_func(reduction=reduction)
        self.to(self.device)

    def forward(self, s):
        self._engine_sync()
        return self.fc_out(self.net(s))

    def actions(self, obses):
        na = self._native_act()
        if na is not None:
            return self._act_gpu(obses, na)
        obses_t = T.as_tensor(obses, dtype=T.float32).to(self.device)
        q_values = self(obses_t)
        return T.argmax(q_values, dim=1).detach().tolist()


class DuelingDeepQNetwork(Network):
    """R:dqn/network.py:77-117.  Acting uses the advantage stream only (:110-117)."""

    def __init__(self, device, lr, nn_conf_func, input_dim, output_dim, reduction='mean'):
        super().__init__(device, nn_conf_func, input_dim)
        self.fc_val = nn.Linear(self.fc_out_dim, 1)
        self.fc_adv = nn.Linear(self.fc_out_dim, output_dim)
        self.aggregate_layer = (lambda val, adv: T.add(val, (adv - adv.mean(dim=1, keepdim=True))))
        self.optimizer = self.optim_func(self.parameters(), lr=lr)
        self.loss = self.loss_func(reduction=reduction)
        self.to(self.device)

    def forward(self, s):
        self._engine_sync()
        net = self.net(s)
        return self.aggregate_layer(self.fc_val(net), self.fc_adv(net))

    def value(self, s):
        self._engine_sync()
        return self.fc_val(self.net(s))

    def advantages(self, s):
        self._engine_sync()
        return self.fc_adv(self.net(s))

    def actions(self, obses):
        na = self._native_act()
        if na is not None:
            return self._act_gpu(obses, na)
        obses_t = T.as_tensor(obses, dtype=T.float32).to(self.device)
        adv_q_values = self.advantages(obses_t)
        return T.argmax(adv_q_values, dim=1).detach().tolist()
