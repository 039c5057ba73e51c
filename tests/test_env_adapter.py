"""CPU: dqn.env_adapter.GymnasiumVecEnv -- gymnasium 5-tuple envs behind the vectorised API of
R:train.py's loop, with the baselines wrappers' semantics (auto-reset, time limit, repeat,
Monitor episode info; R:dqn/utils/baselines_wrappers/)."""
import numpy as np
import pytest

from dqn.env_adapter import GymnasiumVecEnv


class ToyEnv:
    """CustomEnvWrapper-shaped (R:dqn/env_wrap.py:69-108): reset -> (obs, info), step -> 5-tuple;
    the episode terminates after `length` steps; info carries the wrapper's "r" / "l"."""

    def __init__(self, length=3, dim=4, seed=0):
        self.length, self.dim = length, dim
        self.rng = np.random.default_rng(seed)
        self.resets = 0

    def reset(self, *, seed=None, options=None):
        self.t, self.total = 0, 0.0
        self.resets += 1
        return np.full(self.dim, -float(self.resets), np.float32), {"l": 0, "r": 0.0}

    def step(self, action):
        self.t += 1
        rew = float(action) + 0.5
        self.total += rew
        obs = np.full(self.dim, float(self.t), np.float32)
        return obs, rew, self.t >= self.length, False, {"l": self.t, "r": self.total}


def test_reset_and_autoreset_store_the_reset_observation():
    env = GymnasiumVecEnv([lambda: ToyEnv(length=2)])
    o = env.reset()
    assert o.shape == (1, 4) and o.dtype == np.float32 and o[0, 0] == -1
    o, r, d, infos = env.step([1])
    assert o[0, 0] == 1 and r[0] == 1.5 and not d[0]
    o, r, d, infos = env.step([0])
    # terminal step: done, and (DummyVecEnv) the slot holds the NEXT episode's reset obs
    assert d[0] and o[0, 0] == -2
    assert infos[0]["l"] == 2 and infos[0]["r"] == 2.0            # the wrapper's counters
    assert infos[0]["episode"]["l"] == 2 and infos[0]["episode"]["r"] == 2.0   # Monitor


def test_time_limit_and_repeat():
    env = GymnasiumVecEnv([lambda: ToyEnv(length=100)], max_episode_steps=3, repeat=2)
    env.reset()
    for t in range(3):
        o, r, d, infos = env.step([1])
        assert r[0] == 3.0                                        # 2 repeats x 1.5
    assert d[0] and infos[0]["TimeLimit.truncated"]


def test_vectorised_envs_and_action_count():
    env = GymnasiumVecEnv([lambda s=s: ToyEnv(length=2 + s, seed=s) for s in range(3)])
    assert env.reset().shape == (3, 4)
    o, r, d, infos = env.step([0, 1, 2])
    assert r.tolist() == [0.5, 1.5, 2.5] and len(infos) == 3
    with pytest.raises(ValueError):
        env.step([0, 1])


def test_old_gym_four_tuple_env_also_works():
    class Old(ToyEnv):
        def reset(self, **kw):
            return super().reset()[0]

        def step(self, a):
            o, r, term, trunc, info = super().step(a)
            return o, r, term, info
    env = GymnasiumVecEnv([lambda: Old(length=1)])
    assert env.reset()[0, 0] == -1
    o, r, d, infos = env.step([0])
    assert d[0] and o[0, 0] == -2
