"""Drop-in `dqn.agent`: the reference's four agents (R:dqn/agent.py:18-320), with
`learn()` running on the MI355X learn engine (libdqnx).

The same class names, constructor keywords and public methods are kept, so `train.py`'s
`getattr(Agents, args.algo)(...)` works unchanged.  The methods are `learn`,
`store_transitions`, `choose_actions`, `epsilon`, `update_target_network`, `load_model`,
`save_model`, `log`, `info_mean` and `transitions_to_tensor`.

What changes underneath:

* The replay memory is the engine's HBM ring (+ SumTree for PER).
* Both networks' parameters are views into the engine's flat parameter buffers.
* The Adam moments live in the engine.
* `learn()` is one stream-ordered launch sequence: sample → gather → forwards → TD → loss →
  backward → Adam.

Host-visible semantics are the reference's, synchronously from the caller's view:

* RNG.  The device sampler draws the minibatch bit-exactly from the caller's global generator:
  CPython's `random` (`random.sample`, uniform replay) or numpy's legacy global state
  (`np.random.uniform`, PER).  learn() stages the current state for the device and advances the
  global generator on the host by exactly the words that draw consumes before it returns
  (dqnx_rng_sample_words: the rejection / duplicate redraws are walked on the host; PER: 2 words
  per sample), so `choose_actions`' epsilon-greedy draws -- or any other host draw -- interleave
  exactly as in the reference.  The state the device returns is checked against that mirror.
* Weights.  `online_network(x)`, `.value` / `.advantages`, `.parameters()` / `named_parameters()`,
  `state_dict()` and every replay / engine read launch a recorded step first; stream order does the
  rest, so they read the post-step weights.
* Errors.  learn() with fewer stored transitions than `batch_size` raises ValueError as
  `random.sample` does (R:dqn/replay_memory.py:39); a sticky device error (PER tree hand-off, empty
  SumTree) comes back with the control block after each step and is raised at the agent's next
  synchronisation point (`choose_actions`, `log`, `save_model`, `flush`).

The train.py loop (R:train.py:88-108: choose_actions -> store_transitions -> learn ->
update_target_network -> log -> save_model) costs one library call per agent method: learn() stages
the RNG state and launches the step at once (dqnx_agent_stage_rng / dqnx_agent_launch: upload, learn
step, control block back, no host wait), so the GPU runs it under update_target_network's and the
next choose_actions' host work; update_target_network() enqueues the soft update; choose_actions runs
the acting launch with host obs / actions (dqnx_act_host) and checks the control block the step sent
back.  DQNX_AGENT_DEFER=1 instead records learn() and has update_target_network() launch it with the
soft update fused into the Adam pass.
"""
from __future__ import annotations

import array
import ctypes
import os
import random
import time
from collections import deque
from datetime import timedelta

import numpy as np
import torch as T

from . import _capi as C
from .engine import LearnEngine, raise_device_error, spec_from_body
from .network import DeepQNetwork, DuelingDeepQNetwork
from .replay_memory import ReplayMemoryNaive, ReplayMemoryPrioritized


def _summary_writer(log_dir):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(log_dir)
    except Exception:   # tensorboard is optional: logging is out of the hot path
        class _Null:
            def add_scalar(self, *a, **k):
                pass

            def close(self):
                pass
        return _Null()


def _cpython_mt_addresses():
    """(state address, position address) of the global generator's MT19937 inside CPython's
    RandomObject (`PyObject_HEAD; int index; uint32_t state[624]`, Modules/_randommodule.c), or None
    when that layout cannot be confirmed against random.getstate() (then learn() takes getstate() +
    dqnx_agent_stage_rng + getrandbits instead: the same draw, ~25 us more host time).  The
    generator object is never moved or freed (random._inst lives as long as the module)."""
    if os.environ.get("DQNX_AGENT_MT_INPLACE", "1") == "0":
        return None
    try:
        import ctypes
        import sys

        import _random
        inst = random._inst
        if sys.implementation.name != "cpython" or not isinstance(inst, _random.Random):
            return None
        head = object.__basicsize__
        if _random.Random.__basicsize__ < head + 4 + 624 * 4:
            return None
        base = id(inst)
        pos = ctypes.c_int32.from_address(base + head)
        mt = (ctypes.c_uint32 * 624).from_address(base + head + 4)
        ref = inst.getstate()[1]
        if pos.value != ref[624] or tuple(mt) != ref[:624]:
            return None
        return base + head + 4, base + head
    except Exception:   # any doubt: the portable path
        return None


def _raw_stream(device_index):
    """The current HIP stream of the device, as dqn.engine.LearnEngine.stream() takes it (torch's current
    stream), without building a torch Stream object per call."""
    return T._C._cuda_getCurrentRawStream(device_index)


def _interp2(x, x1, f0, f1):
    """np.interp(x, [0, x1], [f0, f1]) for a scalar x, bit for bit (numpy's arr_interp: left / right
    values outside the points, else slope * (x - xp[0]) + fp[0] in float64), without the ~3 us of
    array conversions per call (epsilon() runs once per env per choose_actions).
    tests/test_shim.py checks it against np.interp."""
    x = float(x)
    if x >= x1:
        return float(f1)
    if x <= 0.0:
        return float(f0)
    return (float(f1) - float(f0)) / (float(x1) - 0.0) * (x - 0.0) + float(f0)


def _obs_dim(input_dim) -> int:
    shape = getattr(input_dim, "shape", None)
    if shape is not None:
        return int(np.prod(shape))
    return int(input_dim)


def _per_numpy121() -> bool:
    """The SumTree arithmetic the reference would run with under THIS interpreter's numpy: the
    reference's float32 priorities make `change` and the ancestor sums float32 under numpy < 2's
    value-based casting (its pinned 1.21) and float64 under numpy >= 2 (NEP 50).
    DQNX_PER_NUMPY121=0/1 overrides."""
    v = os.environ.get("DQNX_PER_NUMPY121")
    if v is not None:
        return v not in ("", "0")
    return int(np.__version__.split(".")[0]) < 2


def _check_optim_loss(network):
    """The engine implements torch.optim.Adam (default betas / eps, no weight decay, no amsgrad)
    and nn.SmoothL1Loss (beta 1).  network_config may name others (R:env/custom_env/macro with
    lane/dqn_config.py:96, 101 lists RMSprop and MSELoss): refuse them instead of silently
    training with a different update rule."""
    opt, loss = network.optimizer, network.loss
    if type(opt) is not T.optim.Adam:
        raise NotImplementedError(f"libdqnx trains with torch.optim.Adam only, got {type(opt).__name__}")
    g = opt.param_groups[0]
    if (tuple(g["betas"]) != (0.9, 0.999) or g["eps"] != 1e-8 or g["weight_decay"] != 0 or g["amsgrad"]
            or g.get("maximize", False)):
        raise NotImplementedError("libdqnx implements Adam with its defaults (betas (0.9, 0.999), eps 1e-8, "
                                  "weight_decay 0, amsgrad off)")
    if type(loss) is not T.nn.SmoothL1Loss or getattr(loss, "beta", 1.0) != 1.0:
        raise NotImplementedError(f"libdqnx trains with nn.SmoothL1Loss(beta=1) only, got {loss!r}")


class Agent:
    """R:dqn/agent.py:18-147."""

    _network_cls = None
    _reduction = "mean"

    def __init__(self, n_env, lr, gamma, epsilon_start, epsilon_min, epsilon_decay, epsilon_exp_decay, nn_conf_func,
                 input_dim, output_dim, batch_size, min_buffer_size, buffer_size, update_target_frequency,
                 target_soft_update, target_soft_update_tau, save_frequency, log_frequency, save_dir, log_dir, load,
                 algo, gpu):
        self.n_env = n_env
        self.lr = lr
        self.gamma = gamma
        self.epsilon_start = epsilon_start
        self.epsilon_min = epsilon_min
        self.epsilon_decay = epsilon_decay
        self.epsilon_exp_decay = epsilon_exp_decay
        self.nn_conf_func = nn_conf_func
        self.input_dim = input_dim
        self.output_dim = output_dim
        self.batch_size = batch_size
        self.min_buffer_size = min_buffer_size
        self.buffer_size = buffer_size
        self.update_target_frequency = update_target_frequency
        self.target_soft_update = target_soft_update
        self.target_soft_update_tau = target_soft_update_tau
        self.save_frequency = save_frequency
        self.log_frequency = log_frequency
        self.load = load

        self.step = 0
        self.resume_step = 0
        self.episode_count = 0
        self.ep_info_buffer = deque([], maxlen=50)

        path = algo + '_lr' + str(lr)
        self.save_path = save_dir + path + '_' + 'model.pack'
        self.summary_writer = _summary_writer(log_dir + path + '/')

        if not T.cuda.is_available():
            raise RuntimeError("the dqn learn engine needs a ROCm GPU (MI355X); there is no CPU path")
        self.device = T.device("cuda:" + str(gpu))
        self.start_time = time.time()
        self.algo = algo
        self._build()

    # -- composition (R:dqn/agent.py:275-320) ------------------------------------------
    def _build(self):   # noqa: C901
        cls = type(self)._network_cls
        # same construction order as the reference: online, then target (torch RNG stream)
        self.online_network = cls(self.device, self.lr, self.nn_conf_func, self.input_dim, self.output_dim,
                                  reduction=self._reduction)
        self.target_network = cls(self.device, self.lr, self.nn_conf_func, self.input_dim, self.output_dim,
                                  reduction=self._reduction)
        _check_optim_loss(self.online_network)
        spec = spec_from_body(self.online_network.net, _obs_dim(self.input_dim), self.output_dim,
                              dueling=cls is DuelingDeepQNetwork)
        self.engine = LearnEngine(spec, type(self).__name__, self.batch_size, self.buffer_size, gamma=self.gamma,
                                  lr=self.lr, tau=self.target_soft_update_tau, n_env=self.n_env, device=self.device,
                                  eps_dec=self.epsilon_decay,
                                  compute_dtype=os.environ.get("DQNX_COMPUTE_DTYPE", "fp32"),
                                  per_numpy121=_per_numpy121())
        self.online_network.bind_flat(self.engine.param_views(self.engine.params), self.engine.params, spec,
                                      engine=self.engine)
        self.target_network.bind_flat(self.engine.param_views(self.engine.target_params), self.engine.target_params,
                                      spec, engine=self.engine)
        self.replay_memory_buffer = self._make_replay()
        self._learn_steps = 0          # learn() calls since the last log (throughput metric)
        self._learn_t0 = time.time()
        self._defer = os.environ.get("DQNX_AGENT_DEFER", "0") != "0"
        self._mt = self._live_mt()     # learn() stages and advances the live generator in one call
        self._choose_cache = None      # dqnx_agent_choose's arguments, resolved once
        self._eps_logs = None          # (epsilon_start, epsilon_min), np.log of each
        self._learn_pending = False    # learn() recorded, not launched yet (DQNX_AGENT_DEFER=1)
        if os.environ.get("DQNX_AGENT_GRAPHS", "0") == "1":   # each learn step as one graph launch
            self.engine.set_graphs(True)
        self.engine.launch_hook = self._launch_pending
        self.engine.settle_hook = self.flush
        self.update_target_network(force=True)

    def _make_replay(self):
        return ReplayMemoryNaive(self.buffer_size, self.batch_size, engine=self.engine)

    # -- replay ------------------------------------------------------------------------
    def transitions_to_tensor(self, transitions):
        """R:dqn/agent.py:71-78 (API compatibility; learn() gathers on the device)."""
        obses_t = T.as_tensor(np.asarray([t[0] for t in transitions]), dtype=T.float32).to(self.device)
        actions_t = T.as_tensor(np.asarray([t[1] for t in transitions]), dtype=T.int64).to(self.device).unsqueeze(-1)
        rews_t = T.as_tensor(np.asarray([t[2] for t in transitions]), dtype=T.float32).to(self.device).unsqueeze(-1)
        dones_t = T.as_tensor(np.asarray([t[3] for t in transitions]), dtype=T.float32).to(self.device).unsqueeze(-1)
        new_obses_t = T.as_tensor(np.asarray([t[4] for t in transitions]), dtype=T.float32).to(self.device)
        return obses_t, actions_t, rews_t, dones_t, new_obses_t

    def store_transitions(self, obses, actions, rews, dones, new_obses, infos):
        """R:dqn/agent.py:80-84."""
        self._launch_pending()   # a recorded learn step samples the ring as it was at learn()
        for i in self.replay_memory_buffer.store_transitions(obses, actions, rews, dones, new_obses):
            if infos:
                self.ep_info_buffer.append({'r': infos[i]['r'], 'l': infos[i]['l']})
                self.episode_count += 1

    # -- acting (R:dqn/agent.py:86-99) -------------------------------------------------
    def epsilon(self):
        """R:dqn/agent.py:86-90 (called once per env by choose_actions)."""
        if self.epsilon_exp_decay:
            lg = getattr(self, "_eps_logs", None)
            if lg is None or lg[0] != (self.epsilon_start, self.epsilon_min):   # (np.log once per setting)
                lg = self._eps_logs = ((self.epsilon_start, self.epsilon_min), np.log(self.epsilon_start),
                                       np.log(self.epsilon_min))
            return np.exp(_interp2(self.step * self.n_env, self.epsilon_decay, lg[1], lg[2]))
        return _interp2(self.step * self.n_env, self.epsilon_decay, self.epsilon_start, self.epsilon_min)

    def choose_actions(self, obses):
        self._launch_pending()
        fast = self._choose_one_call(obses)
        if fast is not None:
            return fast
        actions = self.online_network.actions(obses)   # (waits for the stream: the learn step ran)
        self._settle(wait=True)                        # free after that wait: errors, RNG mirror check
        for i in range(len(actions)):
            if random.random() <= self.epsilon():
                actions[i] = random.randint(0, self.output_dim - 1)
        return actions

    def _choose_one_call(self, obses):
        """choose_actions as ONE library call (dqnx_agent_choose): the acting kernel on the engine's online
        parameters, the epsilon-greedy draws of R:dqn/agent.py:95-97 on the live `random` generator in
        place (while the kernel runs), the wait (GIL released) and the last learn step's readback checks.
        None when that path does not apply (the generator's layout unconfirmed, a non-MLP body, device
        observations, more than CHOOSE_MAX_ENVS rows): the method-by-method path runs instead."""
        if self._mt is None or isinstance(obses, T.Tensor):
            return None
        x = obses
        if not (isinstance(x, np.ndarray) and x.dtype == np.float32 and x.ndim == 2 and x.flags.c_contiguous):
            x = np.ascontiguousarray(obses, dtype=np.float32)
            if x.ndim != 2:
                x = x.reshape(x.shape[0], -1)
        n = x.shape[0]
        c = self._choose_cache
        if c is None or c[0] < n:
            c = self._choose_cache = self._choose_setup(n)
            if c is None:
                return None
        cap, f, h, mt, pos, out, oaddr, sptr, nbytes, dev = c
        if x.shape[1] != self.engine.spec.obs_dim:
            raise ValueError(f"observations of width {x.shape[1]}, the network takes {self.engine.spec.obs_dim}")
        rc = f(h, x.__array_interface__["data"][0], n, float(self.epsilon()), mt, pos, oaddr, sptr, nbytes,
               C.CHOOSE_GIL_HELD, _raw_stream(dev))
        self.engine._ag_unread = False   # (the call consumed the last step's readback)
        if rc != C.DQNX_OK:
            if rc == C.DQNX_EDEVICE:   # the sticky device error (or the RNG mirror mismatch the message names)
                err = self.engine.ctrl().error
                if err:
                    raise_device_error(err)
                raise RuntimeError("libdqnx: " + C.lib().dqnx_last_error().decode(errors="replace"))
            C.check(rc, "agent_choose")
        return out[:n].tolist()

    def _choose_setup(self, n):
        if n > C.CHOOSE_MAX_ENVS or os.environ.get("DQNX_AGENT_CHOOSE", "1") == "0":
            return None
        net = self.online_network
        na = net._native_act()
        spec = self.engine.spec
        if na is None or spec.kind != C.DQNX_NET_MLP or na[1] is not self.engine.params:
            return None
        L = C.lib()
        desc = spec.to_c()
        cap = min(max(n, 64), C.CHOOSE_MAX_ENVS)
        nb = int(L.dqnx_act_host_scratch_bytes(ctypes.byref(desc), cap))
        if not nb:
            return None
        self._choose_scratch = T.zeros((nb + 15) // 16 * 4, dtype=T.float32, device=self.engine.device)
        out = np.zeros(cap, dtype=np.int32)
        self._choose_out = out
        dev = self.engine.device.index if self.engine.device.index is not None else T.cuda.current_device()
        return (cap, L.dqnx_agent_choose, self.engine.h, self._mt[0], self._mt[1], out,
                out.__array_interface__["data"][0], self._choose_scratch.data_ptr(), self._choose_scratch.numel() * 4,
                dev)

    # -- learning ----------------------------------------------------------------------
    def _check_population(self):
        """random.sample(deque, batch_size) raises when the deque is shorter (R:dqn/replay_memory.py:39)."""
        if self.engine.ring_size < self.batch_size:
            raise ValueError("Sample larger than population or is negative")

    def _live_mt(self):
        return _cpython_mt_addresses()

    def _rng_handoff(self):
        """Stage the global state for the device's draw and move the global generator past it now
        (dqnx_agent_stage_rng: the words random.sample consumes, walked on the host)."""
        words = self.engine.agent_stage_rng(C.DQNX_RNG_PY, array.array("I", random.getstate()[1]))
        random.getrandbits(32 * words)   # exactly `words` MT19937 outputs, gauss_next untouched

    def _pre_learn(self):
        """Per-algorithm host bookkeeping before the step is launched (PER: the beta step)."""

    def _launch_learn(self, soft_update):
        self._pre_learn()
        self.engine.agent_launch(soft_update=soft_update)   # RNG upload, learn step, control block back
        self._learn_pending = False

    def _launch_pending(self, soft_update=False):
        if self._learn_pending:
            self._launch_learn(soft_update)

    def _settle(self, wait):
        """Look at the control block the last launched step sent back (if it has arrived, or waiting
        for it): raises its sticky device error, and a difference between the device sampler's
        advanced state and the host mirror learn() installed."""
        self.engine.agent_readback(wait)

    def flush(self):
        """Launch a recorded learn step, wait for it and raise any device error it reported.  Not
        needed for correctness (every read launches a recorded step first); agent methods that
        synchronise anyway call it."""
        self._launch_pending()
        self._settle(wait=True)

    def learn(self):
        """One learn step on the engine (R:dqn/agent.py:166-185 / 204-226 / 245-272): launched at once
        (DQNX_AGENT_DEFER=1: recorded and launched by the next agent call, update_target_network()
        fusing its soft update into the step's Adam pass)."""
        self._launch_pending()
        self._settle(wait=False)
        self._check_population()
        self._count_learn()
        if self._mt is not None:   # one call: stage + advance random._inst in place (+ launch)
            self.engine.agent_learn_mt(self._mt[0], self._mt[1], launch=not self._defer)
            self._learn_pending = self._defer
            return
        self._rng_handoff()
        if self._defer:
            self._learn_pending = True
        else:
            self._launch_learn(soft_update=False)

    def _count_learn(self):
        self._learn_steps += 1

    def learn_throughput(self):
        """Sampled transitions per second through learn() since the last call (the metric
        SURVEY.md §5 adds at log cadence; host clock, no extra device sync)."""
        now = time.time()
        dt = now - self._learn_t0
        rate = self._learn_steps * self.batch_size / dt if dt > 0 else 0.0
        self._learn_steps, self._learn_t0 = 0, now
        return rate

    def update_target_network(self, force=False):
        """R:dqn/agent.py:101-110.  Right after learn() (train.py's order) the soft update rides in
        the learn step's Adam pass (DQNX_STEP_SOFT_UPDATE: the same arithmetic, bitwise)."""
        hard = (not self.target_soft_update and self.step % (self.update_target_frequency // self.n_env) == 0) or force
        if self._learn_pending and self.target_soft_update and not hard:
            self._launch_learn(soft_update=True)
            return
        self._launch_pending()
        if hard:
            self.engine.hard_update()
        elif self.target_soft_update:
            self.engine.soft_update()

    # -- checkpoints / logging (R:dqn/agent.py:112-147) ---------------------------------
    def load_model(self):
        import os
        self.flush()
        if self.load and os.path.exists(self.save_path):
            print()
            print("Resume training from " + self.save_path + "...")
            self.resume_step, self.episode_count, rew_mean, len_mean = self.online_network.load(self.save_path)
            [self.ep_info_buffer.append({'r': rew_mean, 'l': len_mean})
             for _ in range(np.min([self.episode_count, self.ep_info_buffer.maxlen]))]
            print("Step: ", self.resume_step * self.n_env, ", Episodes: ", self.episode_count, ", Avg Rew: ",
                  rew_mean, ", Avg Ep Len: ", len_mean)
            self.update_target_network(force=True)
            self.step = self.resume_step

    def save_model(self):
        if self.step % self.save_frequency == 0 and self.step > self.resume_step:
            self.flush()
            print()
            print("Saving model...")
            T.cuda.synchronize(self.device)
            self.online_network.save(self.save_path, self.step, self.episode_count, self.info_mean('r'),
                                     self.info_mean('l'))
            print("OK!")

    def log(self):
        if self.step % self.log_frequency == 0 and self.step > self.resume_step:
            self.flush()
            rew_mean, len_mean = self.info_mean('r'), self.info_mean('l')
            print()
            print('Step: ', self.step * self.n_env, ' (' + str(self.step) + 'x' + str(self.n_env) + ')')
            print('Avg Rew: ', rew_mean)
            print('Avg Ep Len: ', len_mean)
            print('Episodes: ', self.episode_count)
            print('---', str(timedelta(seconds=round((time.time() - self.start_time), 0))), '---')
            self.summary_writer.add_scalar('AvgRew', rew_mean, global_step=self.step * self.n_env)
            self.summary_writer.add_scalar('AvgEpLen', len_mean, global_step=self.step * self.n_env)
            self.summary_writer.add_scalar('Episodes', self.episode_count, global_step=self.step * self.n_env)
            self.summary_writer.add_scalar('Loss', self.engine.loss(), global_step=self.step * self.n_env)
            self.summary_writer.add_scalar('LearnTransitionsPerSec', self.learn_throughput(),
                                           global_step=self.step * self.n_env)

    def info_mean(self, i):
        i_mean = np.mean([e[i] for e in self.ep_info_buffer])
        return i_mean if not np.isnan(i_mean) else 0.0


class SimpleAgent(Agent):
    """R:dqn/agent.py:150-185 (vanilla DQN target: max over the target network)."""


class DoubleAgent(Agent):
    """R:dqn/agent.py:188-226 (Double DQN target)."""


class PerDoubleAgent(Agent):
    """R:dqn/agent.py:229-272 (prioritised replay, IS-weighted Huber)."""

    _reduction = "none"

    def _make_replay(self):
        return ReplayMemoryPrioritized(self.buffer_size, self.batch_size, self.epsilon_decay, engine=self.engine)

    def _check_population(self):
        # the reference samples a partly filled tree (with repeats); an empty one has no transitions
        if self.engine.ring_size == 0:
            raise ValueError("PER sample from an empty replay memory")

    def _live_mt(self):
        return None   # numpy's generator feeds the PER draw (and _pre_learn runs at the launch)

    def _rng_handoff(self):
        """np.random.uniform once per sample (R:dqn/replay_memory.py:79-80): 2 words each."""
        st = np.random.get_state()
        buf = np.empty(625, dtype=np.uint32)
        buf[:624] = st[1]
        buf[624] = st[2]
        self.engine.agent_stage_rng(C.DQNX_RNG_NP, buf)
        np.random.random_sample(self.batch_size)   # the same 2 * batch_size legacy MT19937 words

    def learn(self):
        self._launch_pending()                            # a step recorded earlier keeps its own step
        self._learn_step_at = self.step * self.n_env      # R:dqn/agent.py:247 (the step of THIS learn)
        super().learn()

    def _pre_learn(self):
        e = self.engine
        if self._learn_step_at != e.agent_step:           # any other sampler call moved it too
            e.set_agent_step(self._learn_step_at)


class DQNAgent(SimpleAgent):
    """R:dqn/agent.py:275-284."""
    _network_cls = DeepQNetwork


class DoubleDQNAgent(DoubleAgent):
    """R:dqn/agent.py:287-296."""
    _network_cls = DeepQNetwork


class DuelingDoubleDQNAgent(DoubleAgent):
    """R:dqn/agent.py:299-308."""
    _network_cls = DuelingDeepQNetwork


class PerDuelingDoubleDQNAgent(PerDoubleAgent):
    """R:dqn/agent.py:311-320."""
    _network_cls = DuelingDeepQNetwork
