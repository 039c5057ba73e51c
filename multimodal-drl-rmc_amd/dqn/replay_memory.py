"""Drop-in `dqn.replay_memory` over the learn engine's HBM replay ring
(R:dqn/replay_memory.py:8-98).

The replay content lives on the GPU (ring + SumTree in the engine arena).  These classes
keep the reference's API:

* `store_transitions(...)` — a generator yielding the env indices whose transition is
  terminal, as the reference does;
* `sample_transitions(step)`;
* `update_batch_priorities(tree_indices, abs_td_errors_np)`;
* a `replay_buffer` attribute.

`Agent.learn()` never calls `sample_transitions`: the engine samples, gathers and learns in
one stream-ordered step.  The host-side `sample_transitions` exists for API compatibility
and tests. It returns the same positions and RNG advance as the reference, with the rows
copied back to the host.
"""
from __future__ import annotations

import random

import numpy as np
import torch


class RingView:
    """Read-only deque-like view of the engine's replay ring (logical order, 0 = oldest)."""

    def __init__(self, engine):
        self.engine = engine

    def __len__(self):
        return self.engine.ring_size

    @property
    def maxlen(self):
        return self.engine.capacity

    def slot(self, i: int) -> int:
        n = len(self)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError("deque index out of range")
        return (self.engine.ring_wptr - n + i) % self.engine.capacity

    def rows(self, slots):
        e = self.engine
        e.launch_recorded()
        s = torch.as_tensor(np.asarray(slots, dtype=np.int64), device=e.device)
        D = e.spec.obs_dim
        obs = e.ring_obs.index_select(0, s)[:, :D].cpu().numpy()
        nobs = e.ring_next_obs.index_select(0, s)[:, :D].cpu().numpy()
        act = e.ring_act.index_select(0, s).cpu().numpy()
        rew = e.ring_rew.index_select(0, s).cpu().numpy()
        done = e.ring_done.index_select(0, s).cpu().numpy()
        return [(obs[j], int(act[j]), float(rew[j]), bool(done[j]), nobs[j]) for j in range(len(slots))]

    def __getitem__(self, i):
        return self.rows([self.slot(i)])[0]

    def __iter__(self):
        return iter(self.rows([self.slot(i) for i in range(len(self))]))


class SumTreeView:
    """Read-only view of the engine's SumTree with the reference's attribute names
    (R:dqn/utils/sum_tree.py:4-73)."""

    def __init__(self, engine):
        self.engine = engine
        self.capacity = engine.capacity

    @property
    def tree(self) -> np.ndarray:
        self.engine.launch_recorded()
        return self.engine.sumtree.cpu().numpy()

    @property
    def size(self):
        return self.engine.ring_size

    @property
    def data_pointer(self):
        return self.engine.ring_wptr

    @property
    def max_priority_index(self):
        return int(self.engine.ctrl().per_max_idx)

    @property
    def min_priority_index(self):
        return int(self.engine.ctrl().per_min_idx)

    @property
    def total_priority(self):
        return float(self.engine.sumtree[0].item())

    @property
    def max_priority(self):
        return float(self.engine.sumtree[self.max_priority_index].item())

    @property
    def min_priority(self):
        return float(self.engine.sumtree[self.min_priority_index].item())

    def __len__(self):
        return self.size


class ReplayMemory:
    """R:dqn/replay_memory.py:8-21."""

    def __init__(self, buffer_size, batch_size, engine=None):
        if engine is None:
            raise RuntimeError("the GPU replay memory lives in a learn engine: construct it through an agent "
                               "(dqn.agent.*Agent) or pass engine=")
        self.batch_size = batch_size
        self.buffer_size = buffer_size
        self.engine = engine

    def store_transitions(self, obses, actions, rews, dones, new_obses):
        """Push the n_env transitions (host arrays) and yield the indices whose `done` is set
        (R:dqn/replay_memory.py:30-36 / 56-67)."""
        n = len(actions)
        self.engine.launch_recorded()   # a recorded learn step samples the ring as it was at learn()
        if n:
            self.engine.push_host(obses, actions, rews, dones, new_obses, n)
        for e, done in enumerate(dones):
            if done:
                yield e

    def sample_transitions(self, step=None):
        raise NotImplementedError


class ReplayMemoryNaive(ReplayMemory):
    """R:dqn/replay_memory.py:24-39."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.replay_buffer = RingView(self.engine)

    def sample_transitions(self, step=None):
        # random.sample over a sequence only uses its length to draw positions, so sampling
        # range(len) consumes the global stream exactly like sampling the deque
        self.engine.settle()
        pos = random.sample(range(len(self.replay_buffer)), self.batch_size)
        return self.replay_buffer.rows([self.replay_buffer.slot(p) for p in pos])


class ReplayMemoryPrioritized(ReplayMemory):
    """R:dqn/replay_memory.py:43-98 (device SumTree, see csrc/per.hip)."""

    def __init__(self, buffer_size, batch_size, eps_dec, engine=None):
        super().__init__(buffer_size, batch_size, engine=engine)
        self.replay_buffer = SumTreeView(self.engine)
        c = self.engine.cfg
        self.epsilon = c.per_eps
        self.alpha = c.per_alpha
        self.beta_start = c.per_beta_start
        self.beta_end = c.per_beta_end
        self.beta_inc = eps_dec
        self.max_priority_high = c.per_max_priority

    def sample_transitions(self, step):
        """(is_weights, tree_indices, transitions) drawn from numpy's global RandomState,
        which is advanced exactly as the reference's np.random.uniform calls would."""
        e = self.engine
        e.settle()
        e.set_np_state_from_global()
        e.set_agent_step(int(step))
        e.per_sample()
        e.get_np_state_to_global()
        slots = e.batch_idx.cpu().numpy().astype(np.int64)
        isw = e.is_weights.cpu().numpy().astype(np.float64)
        tree_indices = (slots + e.capacity - 1).tolist()
        return list(isw), tree_indices, self.replay_buffer_rows(slots)

    def replay_buffer_rows(self, slots):
        return RingView(self.engine).rows(slots)

    def update_batch_priorities(self, tree_indices, abs_td_errors_np):
        e = self.engine
        e.launch_recorded()
        slots = torch.as_tensor(np.asarray(tree_indices, dtype=np.int64) - (e.capacity - 1), dtype=torch.int32)
        absd = torch.as_tensor(np.asarray(abs_td_errors_np, dtype=np.float32).reshape(-1))
        e.per_update_priorities(slots, absd)
