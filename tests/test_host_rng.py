"""CPU: the host RNG mirror of the drop-in Agent (include/dqnx.h dqnx_rng_sample_words /
dqnx_rng_advance, csrc/host_rng.cpp).  No GPU: host-only entry points of libdqnx.

learn() advances the caller's global generator by the words the device's draw consumes, so it must
agree with the reference's own draw exactly: CPython's random.sample over the deque
(R:dqn/replay_memory.py:38-39) in both of its branches, and numpy's legacy uniform
(R:dqn/replay_memory.py:79-80, two MT19937 words per sample)."""
import random

import numpy as np
import pytest

from dqn import _capi as C
from dqn.engine import LearnEngine


class _Mirror:   # the two host-only methods, without constructing an engine (which needs a GPU)
    L = C.lib()
    sample_words = LearnEngine.sample_words
    rng_advance = LearnEngine.rng_advance


M = _Mirror()


def _state():
    return np.asarray(random.getstate()[1], dtype=np.uint32)


@pytest.mark.parametrize("n,k", [
    (1, 1), (5, 5), (21, 3), (26, 6), (100, 32), (85, 6), (86, 6),   # pool branch / its threshold
    (300, 32), (1000, 32), (700, 64), (5000, 256), (20000, 1024), (1_000_000, 1024),
    (4096, 4096), (5000, 4096), (1_000_000, 4096), (100_000, 8192), (2 ** 31 - 1, 64),
])
def test_sample_words_match_cpython(n, k):
    random.seed(n * 7919 + k)
    for _ in range(3):   # successive draws, from states at any position in the block
        s0 = _state()
        words, after = M.sample_words(s0, n, k)
        random.sample(range(n), k)
        assert np.array_equal(after, _state()), (n, k)
        # getrandbits(32 * words) moves a state by exactly the same words: what learn() runs
        v, _, g = random.getstate()
        random.setstate((v, tuple(int(x) for x in s0), g))
        random.getrandbits(32 * words)
        assert np.array_equal(after, _state()), (n, k, words)
        random.random()   # move on by one word


def test_sample_words_refuses_oversized_sample():
    s0 = _state()
    with pytest.raises(C.DqnxError, match="Sample larger than population"):
        C.check(C.lib().dqnx_rng_sample_words(s0.ctypes.data, 10, 32, None,
                                              C.ctypes.byref(C.I64())), "rng_sample_words")


@pytest.mark.parametrize("k", [1, 32, 311, 312, 1024, 8192])
def test_rng_advance_matches_numpy_legacy_uniform(k):
    np.random.seed(k)
    np.random.uniform(size=k % 7)   # any starting position
    st = np.random.get_state()
    s0 = np.append(np.asarray(st[1], dtype=np.uint32), np.uint32(st[2]))
    after = M.rng_advance(s0, 2 * k)
    for i in range(k):   # the reference's per-sample uniform(low, high) calls
        np.random.uniform(i, i + 1)
    st = np.random.get_state()
    assert np.array_equal(after, np.append(np.asarray(st[1], dtype=np.uint32), np.uint32(st[2])))


def test_cpython_generator_layout_and_in_place_advance():
    """The drop-in's dqnx_agent_learn_mt works on random._inst's own MT19937 words (checked against
    random.getstate() by dqn.agent._cpython_mt_addresses).  Writing the mirrored post-draw state there
    leaves the generator exactly where random.sample(range(n), k) leaves it."""
    import ctypes

    from dqn.agent import _cpython_mt_addresses
    addr = _cpython_mt_addresses()
    assert addr is not None, "CPython RandomObject layout not recognised (the agent falls back to getstate)"
    mt = (ctypes.c_uint32 * 624).from_address(addr[0])
    pos = ctypes.c_int32.from_address(addr[1])
    for n, k in ((1000, 32), (1_000_000, 1024), (5000, 4096)):
        random.seed(n + k)
        random.random()
        s0 = random.getstate()
        s625 = np.append(np.frombuffer(mt, dtype=np.uint32), np.uint32(pos.value))
        assert np.array_equal(s625, np.asarray(s0[1], dtype=np.uint32))
        _, after = M.sample_words(s625, n, k)
        ctypes.memmove(mt, after.ctypes.data, 624 * 4)   # what dqnx_agent_learn_mt writes back
        pos.value = int(after[624])
        moved = random.getstate()
        random.setstate(s0)
        random.sample(range(n), k)
        assert moved == random.getstate(), (n, k)
        assert moved[2] == s0[2]   # gauss_next untouched
