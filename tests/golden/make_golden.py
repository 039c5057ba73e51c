#!/usr/bin/env python3
"""Generate golden fixtures by running the REFERENCE itself (build container only).

Imports /root/reference (youcefMehamlia/Multimodal-DRL-RMC) read-only with the stubs
SURVEY.md §8(c) lists (colorama, torch.utils.tensorboard; dqn/ and env/ package
__init__ bypassed because they import gymnasium/traci), drives the reference's own
agents / replay memories / SumTree on seeded synthetic transitions, and writes small
.npz files of inputs and outputs to tests/golden/.  Nothing from the reference's
source is copied: the fixtures are data (seeds, RNG states, indices, losses,
parameter tensors).

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

Fixture inputs that are large (replay contents, initial weights) are regenerated on
the GPU box from seeds (oracle.ref.synth_transitions / oracle.ref.reference_init);
each fixture stores a SHA-256 of those regenerated inputs so a mismatch is caught.
"""
import hashlib
import importlib
import importlib.util
import os
import random
import sys
import types
from collections import OrderedDict

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import ref as O  # noqa: E402  (synthetic data + init are shared with the tests)


def _stub_modules():
    col = types.ModuleType("colorama")

    class _C:
        def __getattr__(self, k):
            return ""
    col.Fore = _C()
    col.Style = _C()
    sys.modules["colorama"] = col
    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:
        def __init__(self, *a, **k):
            pass

        def add_scalar(self, *a, **k):
            pass
    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb
    for name, path in (("dqn", "dqn"), ("env", "env"), ("env.custom_env", "env/custom_env")):
        m = types.ModuleType(name)
        m.__path__ = [os.path.join(REF, path)]
        sys.modules[name] = m


def load_reference():
    _stub_modules()
    agent = importlib.import_module("dqn.agent")
    replay = importlib.import_module("dqn.replay_memory")
    sumtree = importlib.import_module("dqn.utils.sum_tree")
    cfg = importlib.import_module("env.dqn_config")
    spec = importlib.util.spec_from_file_location(
        "env.mlp_dqn_config", os.path.join(REF, "env/custom_env/macro with lane/dqn_config.py"))
    mlp_cfg = importlib.util.module_from_spec(spec)
    mlp_cfg.__package__ = "env"
    spec.loader.exec_module(mlp_cfg)
    return agent, replay, sumtree, cfg, mlp_cfg


class Box:
    def __init__(self, n):
        self.shape = (n,)


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def state_array(st):
    return np.array(st[1], dtype=np.uint32)


# ---------------------------------------------------------------------------------------
def gen_sampler(replay_mod):
    """ReplayMemoryNaive.sample_transitions (R:dqn/replay_memory.py:38-39) index vectors."""
    cases = []
    for (n, k, seed) in [(50, 32, 1), (200, 32, 2), (4117, 1024, 3), (4118, 1024, 4), (10000, 1024, 5),
                         (100000, 32, 6), (100000, 4096, 7), (1000000, 1024, 8), (1000000, 4096, 9),
                         (1000000, 8192, 10), (16405, 4096, 11), (16406, 4096, 12), (7, 5, 13), (6, 6, 14)]:
        mem = replay_mod.ReplayMemoryNaive(n, k)
        ids = [np.int64(i) for i in range(n)]
        # store one "transition" per position; obs carries its position
        for i in range(n):
            mem.replay_buffer.append((ids[i], 0, 0.0, False, ids[i]))
        random.seed(seed)
        st_in = state_array(random.getstate())
        tr = mem.sample_transitions()
        st_out = state_array(random.getstate())
        idx = np.array([int(t[0]) for t in tr], dtype=np.int64)
        cases.append((n, k, st_in, st_out, idx))
    out = {}
    for j, (n, k, a, b, idx) in enumerate(cases):
        out[f"c{j}_n"] = np.int64(n)
        out[f"c{j}_k"] = np.int64(k)
        out[f"c{j}_state_in"] = a
        out[f"c{j}_state_out"] = b
        out[f"c{j}_idx"] = idx
    out["count"] = np.int64(len(cases))
    np.savez_compressed(os.path.join(HERE, "sampler.npz"), **out)
    print("sampler.npz", len(cases), "cases")


# ---------------------------------------------------------------------------------------
def gen_np_uniform():
    """numpy legacy uniform draws as used by R:dqn/replay_memory.py:80."""
    np.random.seed(1234)
    st_in = O.np_state_to_array(np.random.get_state())
    lows = np.linspace(0.0, 50.0, 257)
    vals = np.array([np.random.uniform(lows[i], lows[i + 1]) for i in range(256)], dtype=np.float64)
    st_out = O.np_state_to_array(np.random.get_state())
    np.savez_compressed(os.path.join(HERE, "np_uniform.npz"), state_in=st_in, state_out=st_out,
                        lows=lows, vals=vals)
    print("np_uniform.npz")


# ---------------------------------------------------------------------------------------
def make_agent(agent_mod, algo, nn_conf_func, obs_dim, batch, buffer, lr=1e-4, seed=0):
    torch.manual_seed(seed)
    kw = dict(n_env=1, lr=lr, gamma=0.99, epsilon_start=1.0, epsilon_min=0.01, epsilon_decay=2e6,
              epsilon_exp_decay=True, nn_conf_func=nn_conf_func, input_dim=Box(obs_dim), output_dim=8,
              batch_size=batch, min_buffer_size=batch, buffer_size=buffer, update_target_frequency=30000,
              target_soft_update=True, target_soft_update_tau=1e-3, save_frequency=10000,
              log_frequency=4500, save_dir="/tmp/dqnx_golden_save/", log_dir="/tmp/dqnx_golden_log/",
              load=False, algo=algo, gpu="0")
    return getattr(agent_mod, algo)(**kw)


def gen_learn(agent_mod, nn_conf_func, tag, spec_fn, obs_dim, batch, buffer, n_fill, steps, seed,
              algos, full_weights=True, stride=1, full_tree=False):
    for algo in algos:
        ag = make_agent(agent_mod, algo, nn_conf_func, obs_dim, batch, buffer, seed=seed)
        spec = spec_fn(O.algo_spec_head(algo))
        init = O.reference_init(spec, seed)
        sd0 = OrderedDict((k, v.detach().clone()) for k, v in ag.online_network.state_dict().items())
        assert list(sd0.keys()) == list(init.keys()), (list(sd0.keys()), list(init.keys()))
        for k in sd0:
            assert torch.equal(sd0[k], init[k]), k
        obs, act, rew, done, new_obs = O.synth_transitions(n_fill, obs_dim, 8, seed=seed + 100)
        for i in range(n_fill):
            list(ag.replay_memory_buffer.store_transitions(obs[i:i + 1], [int(act[i])], [rew[i]],
                                                           [bool(done[i])], new_obs[i:i + 1]))
        random.seed(seed + 7)
        np.random.seed(seed + 11)
        py_in = state_array(random.getstate())
        np_in = O.np_state_to_array(np.random.get_state())

        # capture losses / sampled positions / PER data per step
        rec = {"loss": [], "pos": [], "isw": [], "absd": []}
        loss_mod = ag.online_network.loss

        def loss_wrap(a, b, _m=loss_mod):
            out = _m(a, b)
            return out
        per = algo.startswith("Per")
        if per:
            orig_sample = ag.replay_memory_buffer.sample_transitions
            orig_update = ag.replay_memory_buffer.update_batch_priorities

            def samp(step, _o=orig_sample):
                w, ti, tr = _o(step)
                rec["pos"].append(np.array(ti, dtype=np.int64))
                rec["isw"].append(np.array(w, dtype=np.float64))
                return w, ti, tr

            def upd(ti, ab, _o=orig_update):
                rec["absd"].append(np.array(ab, dtype=np.float32).reshape(-1))
                return _o(ti, ab)
            ag.replay_memory_buffer.sample_transitions = samp
            ag.replay_memory_buffer.update_batch_priorities = upd
        else:
            buf = ag.replay_memory_buffer.replay_buffer
            ident = {id(t): i for i, t in enumerate(buf)}
            orig_sample = ag.replay_memory_buffer.sample_transitions

            def samp(step=None, _o=orig_sample):
                tr = _o()
                rec["pos"].append(np.array([ident[id(t)] for t in tr], dtype=np.int64))
                return tr
            ag.replay_memory_buffer.sample_transitions = samp
        # loss capture: wrap optimizer.step to read the last computed loss via a hook
        orig_backward = torch.Tensor.backward

        def backward(self, *a, **k):
            rec["loss"].append(float(self.detach()))
            return orig_backward(self, *a, **k)
        torch.Tensor.backward = backward
        try:
            for s in range(steps):
                ag.step = s
                ag.learn()
                ag.update_target_network()
        finally:
            torch.Tensor.backward = orig_backward
        py_out = state_array(random.getstate())
        np_out = O.np_state_to_array(np.random.get_state())
        online = OrderedDict((k, v.detach().clone()) for k, v in ag.online_network.state_dict().items())
        target = OrderedDict((k, v.detach().clone()) for k, v in ag.target_network.state_dict().items())
        opt = ag.online_network.optimizer
        m = OrderedDict()
        v = OrderedDict()
        for (k, p) in ag.online_network.named_parameters():
            st = opt.state[p]
            m[k] = st["exp_avg"].detach().clone()
            v[k] = st["exp_avg_sq"].detach().clone()
        out = dict(algo=np.array(algo), tag=np.array(tag), seed=np.int64(seed), batch=np.int64(batch),
                   buffer=np.int64(buffer), n_fill=np.int64(n_fill), steps=np.int64(steps),
                   obs_dim=np.int64(obs_dim), stride=np.int64(stride),
                   py_state_in=py_in, py_state_out=py_out, np_state_in=np_in, np_state_out=np_out,
                   data_sha=np.array(sha(obs, act, rew, done, new_obs)),
                   init_sha=np.array(sha(*[t.numpy() for t in init.values()])),
                   loss=np.array(rec["loss"], dtype=np.float64),
                   pos=np.stack(rec["pos"]))
        if per:
            out["isw"] = np.stack(rec["isw"])
            out["absd"] = np.stack(rec["absd"])
            tree = ag.replay_memory_buffer.replay_buffer
            out["tree"] = tree.tree.copy() if (full_tree or len(tree.tree) <= 70000) else tree.tree[::stride].copy()
            out["tree_full"] = np.bool_(len(out["tree"]) == len(tree.tree))
            out["tree_max_idx"] = np.int64(tree.max_priority_index)
            out["tree_min_idx"] = np.int64(tree.min_priority_index)
        keys = list(online.keys())
        out["keys"] = np.array(keys)
        for i, k in enumerate(keys):
            for nm, d in (("online", online), ("target", target), ("m", m), ("v", v)):
                t = d[k].reshape(-1).numpy()
                if full_weights and nm in ("online", "target"):
                    out[f"{nm}_{i}"] = t
                else:
                    out[f"{nm}_{i}"] = t[::stride]
                out[f"{nm}_sum_{i}"] = np.float64(t.astype(np.float64).sum())
        fn = os.path.join(HERE, f"learn_{tag}_{algo}.npz")
        np.savez_compressed(fn, **out)
        print(os.path.basename(fn), os.path.getsize(fn), "bytes; losses", rec["loss"])


def gen_sumtree(sumtree_mod):
    """SumTree add/update/get_leaf traces (R:dqn/utils/sum_tree.py) with a non power of two
    capacity, ring wrap-around, duplicate updates and max/min-index rescans."""
    rng = np.random.default_rng(77)
    cap = 1000
    t = sumtree_mod.SumTree(cap)
    ops = []   # (kind, a, b): kind 0=add(priority), 1=update(leaf, priority float32), 2=get_leaf(v)
    outs = []
    for step in range(3000):
        r = rng.random()
        if r < 0.45 or t.size == 0:
            p = t.max_priority if t.max_priority != 0 else 1.0
            if rng.random() < 0.1:
                p = float(np.float32(rng.random()))
            t.add(p, step)
            ops.append((0, -1, float(p)))
            outs.append((t.max_priority_index, t.min_priority_index, float(t.tree[0])))
        elif r < 0.85:
            leaf = int(rng.integers(0, t.size)) + cap - 1
            if rng.random() < 0.3:
                leaf = t.max_priority_index if rng.random() < 0.5 else t.min_priority_index
            p = np.power(np.minimum(np.float32(rng.random() * 1.5) + np.float32(1e-4), np.float32(1.0)),
                         np.float32(0.6)).astype(np.float32)
            t.update(leaf, np.array([p], dtype=np.float32))
            ops.append((1, leaf, float(p)))
            outs.append((t.max_priority_index, t.min_priority_index, float(t.tree[0])))
        else:
            v = float(rng.random() * t.total_priority)
            leaf, p, _ = t.get_leaf(v)
            ops.append((2, -1, v))
            outs.append((leaf, -1, float(p)))
    ops = np.array(ops, dtype=np.float64)
    outs = np.array(outs, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "sumtree.npz"), cap=np.int64(cap), ops=ops, outs=outs,
                        tree=t.tree.copy(), size=np.int64(t.size), ptr=np.int64(t.data_pointer))
    print("sumtree.npz", len(ops), "ops")


def main():
    """python make_golden.py [name ...]: regenerate every fixture, or only the named groups
    (sampler, np_uniform, sumtree, mlp14, mlp284, hybrid284, mlp284b1024, mlp284b4096, mlp284b8192,
    mlp284long1024, mlp284long8192)."""
    only = set(sys.argv[1:])

    def want(name):
        return not only or name in only
    agent_mod, replay_mod, sumtree_mod, cfg, mlp_cfg = load_reference()
    torch.set_num_threads(1)
    if want("sampler"):
        gen_sampler(replay_mod)
    if want("np_uniform"):
        gen_np_uniform()
    if want("sumtree"):
        gen_sumtree(sumtree_mod)
    all_algos = ["DQNAgent", "DoubleDQNAgent", "DuelingDoubleDQNAgent", "PerDuelingDoubleDQNAgent"]
    mlp284 = lambda h: O.mlp_spec(284, 8, h)   # noqa: E731
    if want("mlp14"):
        gen_learn(agent_mod, mlp_cfg.network_config, "mlp14", lambda h: O.mlp_spec(14, 8, h), 14,
                  batch=32, buffer=500, n_fill=300, steps=3, seed=3, algos=all_algos)
    if want("mlp284"):
        gen_learn(agent_mod, mlp_cfg.network_config, "mlp284", mlp284, 284,
                  batch=256, buffer=5000, n_fill=3000, steps=2, seed=5,
                  algos=["DuelingDoubleDQNAgent", "PerDuelingDoubleDQNAgent"])
    if want("hybrid284"):
        gen_learn(agent_mod, cfg.network_config, "hybrid284", lambda h: O.hybrid_spec(8, h), 284,
                  batch=64, buffer=1000, n_fill=600, steps=2, seed=9,
                  algos=["DuelingDoubleDQNAgent"], full_weights=False, stride=37)
    # the bench batch (configs[1]) and the north-star batch (configs[3]'s global minibatch),
    # and configs[4]'s PER batch (fp32 reference arithmetic); weights strided to keep them small
    if want("mlp284b1024"):
        gen_learn(agent_mod, mlp_cfg.network_config, "mlp284b1024", mlp284, 284,
                  batch=1024, buffer=20000, n_fill=20000, steps=2, seed=21,
                  algos=["DuelingDoubleDQNAgent"], full_weights=False, stride=5)
    if want("mlp284b4096"):
        gen_learn(agent_mod, mlp_cfg.network_config, "mlp284b4096", mlp284, 284,
                  batch=4096, buffer=60000, n_fill=60000, steps=2, seed=22,
                  algos=["DuelingDoubleDQNAgent"], full_weights=False, stride=5)
    if want("mlp284b8192"):
        gen_learn(agent_mod, mlp_cfg.network_config, "mlp284b8192", mlp284, 284,
                  batch=8192, buffer=40000, n_fill=40000, steps=2, seed=23,
                  algos=["PerDuelingDoubleDQNAgent"], full_weights=False, stride=5)
    # longer prioritised runs (8 learn steps each, the full SumTree kept): every step's sampled leaves
    # and the final tree pin the engine's float32 priority power over many dependent tree updates
    # (the reference's np.power here is numpy's SVML path; libdqnx computes the correctly rounded powf)
    if want("mlp284long1024"):
        gen_learn(agent_mod, mlp_cfg.network_config, "mlp284long1024", mlp284, 284,
                  batch=1024, buffer=20000, n_fill=20000, steps=8, seed=31,
                  algos=["PerDuelingDoubleDQNAgent"], full_weights=False, stride=5, full_tree=True)
    if want("mlp284long8192"):
        gen_learn(agent_mod, mlp_cfg.network_config, "mlp284long8192", mlp284, 284,
                  batch=8192, buffer=40000, n_fill=40000, steps=8, seed=32,
                  algos=["PerDuelingDoubleDQNAgent"], full_weights=False, stride=5, full_tree=True)


if __name__ == "__main__":
    main()
