"""Gymnasium 5-tuple envs behind the vectorised API the training loop drives.

The reference's HEAD environment wrapper already speaks gymnasium: `CustomEnvWrapper.reset`
returns `(obs, info)` and `step` returns `(obs, rew, terminated, truncated, info)`
(R:dqn/env_wrap.py:69-108).  The vendored baselines wrappers between it and `train.py`
(`MaxEpisodeStepsWrapper`, `Monitor`, `DummyVecEnv`, R:dqn/utils/baselines_wrappers/) still
unpack old-gym 4-tuples and store the raw reset result as an observation, so
`bin/train.sh` fails at its first reset.  `GymnasiumVecEnv` is the replacement for that stack:

* `reset()` -> obs [n_env, D] float32 (R:train.py:69, 86);
* `step(actions)` -> `(new_obs, rews, dones, infos)` (R:train.py:75, 92) with
  `done = terminated or truncated` (or the `max_episode_steps` limit, flagged
  `info["TimeLimit.truncated"]` like MaxEpisodeStepsWrapper), an optional action repeat that
  sums rewards (RepeatActionWrapper), Monitor's `info["episode"] = {"r", "l", "t"}`, and
  DummyVecEnv's auto-reset: a finished env's slot of `new_obs` holds its reset observation
  (R:dqn/utils/baselines_wrappers/dummy_vec_env.py:45-56), exactly what the reference stores.

The infos carry the wrapper's own `"r"` / `"l"` episode counters, which
`Agent.store_transitions` reads for finished episodes (R:dqn/agent.py:80-84).  Pure host
Python: the env loop stays on the CPU (north_star); gymnasium itself is not imported.
"""
from __future__ import annotations

import time
from typing import Callable, List, Sequence

import numpy as np


class GymnasiumVecEnv:
    def __init__(self, env_fns: Sequence[Callable[[], object]], max_episode_steps: int = 0, repeat: int = 0):
        self.envs = [fn() for fn in env_fns]
        self.num_envs = len(self.envs)
        if self.num_envs < 1:
            raise ValueError("need at least one env")
        self.max_episode_steps = int(max_episode_steps)
        self.repeat = int(repeat)
        e0 = self.envs[0]
        self.observation_space = getattr(e0, "observation_space", None)
        self.action_space = getattr(e0, "action_space", None)
        self._elapsed = [0] * self.num_envs
        self._ep_rew = [0.0] * self.num_envs
        self._ep_len = [0] * self.num_envs
        self._t0 = time.time()

    @staticmethod
    def _obs(o) -> np.ndarray:
        return np.asarray(o, dtype=np.float32)

    def _reset_one(self, e: int) -> np.ndarray:
        out = self.envs[e].reset()
        obs = out[0] if isinstance(out, tuple) and len(out) == 2 else out   # gymnasium: (obs, info)
        self._elapsed[e] = 0
        self._ep_rew[e] = 0.0
        self._ep_len[e] = 0
        return self._obs(obs)

    def reset(self) -> np.ndarray:
        return np.stack([self._reset_one(e) for e in range(self.num_envs)])

    def _step_one(self, e: int, action):
        env = self.envs[e]
        total, done, info, obs = 0.0, False, {}, None
        for _ in range(max(1, self.repeat)):   # RepeatActionWrapper: rewards summed, stop at done
            out = env.step(action)
            if len(out) == 5:
                obs, rew, terminated, truncated, info = out
                d = bool(terminated) or bool(truncated)
            else:                                # an old-gym env (4-tuple) works as well
                obs, rew, d, info = out
            total += float(rew)
            if d:
                done = True
                break
        info = dict(info) if info is not None else {}
        self._elapsed[e] += 1
        if self.max_episode_steps > 0 and self._elapsed[e] >= self.max_episode_steps:   # MaxEpisodeStepsWrapper
            done = True
            info["TimeLimit.truncated"] = True
        self._ep_rew[e] += total
        self._ep_len[e] += 1
        if done:                                                                        # Monitor
            info["episode"] = {"r": round(self._ep_rew[e], 6), "l": self._ep_len[e],
                               "t": round(time.time() - self._t0, 6)}
        return self._obs(obs), total, done, info

    def step(self, actions):
        acts: List = list(actions) if np.ndim(actions) else [actions]
        if len(acts) != self.num_envs:
            raise ValueError(f"{len(acts)} actions for {self.num_envs} envs")
        obs, rews, dones, infos = [], np.zeros(self.num_envs, np.float32), np.zeros(self.num_envs, bool), []
        for e in range(self.num_envs):
            o, r, d, info = self._step_one(e, acts[e])
            if d:                                                                       # DummyVecEnv
                o = self._reset_one(e)
            obs.append(o)
            rews[e], dones[e] = r, d
            infos.append(info)
        return np.stack(obs), rews, dones, infos

    def close(self):
        for env in self.envs:
            if hasattr(env, "close"):
                env.close()
