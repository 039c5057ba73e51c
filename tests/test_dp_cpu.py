"""Data-parallel learn step on CPU: world_size 2 over gloo.

`dqn.data_parallel.dp_learn_step` is the exact code bench.py / a DP trainer runs on the GPUs
(RCCL there).  Here it drives an engine stand-in that computes each rank's shard with the
oracle. Two things are checked:
* the decomposition: shard losses scaled by 1/B_global + SUM all-reduce + all-gathered PER
  |delta| reproduce the single-process learn step;
* the collective plumbing.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ref as O

ALGOS = ["DoubleDQNAgent", "PerDuelingDoubleDQNAgent"]


class OracleShardEngine:
    """LearnEngine's DP surface (learn_step(grads_only), grads, per_abs_td, apply_grads)
    computed by the oracle for this rank's shard."""

    def __init__(self, learner, world, rank):
        self.L = learner
        self.world_size, self.rank, self.batch = world, rank, learner.batch_size
        self.keys = list(learner.online)
        self.P = sum(v.numel() for v in learner.online.values())
        self.grads = torch.zeros(self.P + 1)
        self.per_abs_td = torch.zeros(self.batch if learner.per else 0)
        self.rec = None

    def learn_step(self, grads_only=True, soft_update=False):
        from dqn.data_parallel import shard_bounds
        b0, b1 = shard_bounds(self.batch, self.world_size, self.rank)
        self.rec = rec = self.L.learn(shard=(b0, b1))
        self.grads[:self.P] = torch.cat([rec.grads[k].reshape(-1) for k in self.keys])
        self.grads[self.P] = rec.loss
        if self.L.per:
            self.per_abs_td.zero_()
            self.per_abs_td[b0:b1] = torch.from_numpy(rec.abs_td.reshape(-1)[b0:b1])

    def apply_grads(self, soft_update=True):
        g, o = {}, 0
        for k in self.keys:
            n = self.L.online[k].numel()
            g[k] = self.grads[o:o + n].view_as(self.L.online[k])
            o += n
        self.L.apply_grads(g, abs_td=self.per_abs_td.numpy() if self.L.per else None, positions=self.rec.positions)
        if soft_update:
            self.L.update_target_network()
        self.L.step += 1


def make_learner(algo):
    spec = O.mlp_spec(14, 8, O.algo_spec_head(algo))
    L = O.OracleLearner(spec, algo, 32, 500, seed=4, params=O.reference_init(spec, 4), per_pow="cr")
    O.fill_replay(L, *O.synth_transitions(300, 14, 8, seed=104))
    rs = np.random.RandomState(5)
    L.np_state = O.np_state_to_array(rs.get_state())
    import random
    L.py_state = O.py_state_to_array(random.Random(6).getstate())
    return L


def worker(rank, world, port, algo, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from dqn.data_parallel import dp_learn_step
    eng = OracleShardEngine(make_learner(algo), world, rank)
    losses, positions = [], []
    for _ in range(3):
        dp_learn_step(eng, soft_update=True)
        losses.append(float(eng.grads[-1]))
        positions.append(np.asarray(eng.rec.positions))
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), losses=np.array(losses), positions=np.stack(positions),
             **{"on_" + k: v.numpy() for k, v in eng.L.online.items()},
             **{"tg_" + k: v.numpy() for k, v in eng.L.target.items()},
             **({"tree": eng.L.replay.replay_buffer.tree} if eng.L.per else {}))
    dist.destroy_process_group()


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("algo", ALGOS)
def test_dp_world2_matches_single_process(tmp_path, algo):
    mp.spawn(worker, args=(2, free_port(), algo, str(tmp_path)), nprocs=2, join=True)
    ref = make_learner(algo)
    recs = [ref.train_step() for _ in range(3)]
    r0, r1 = (np.load(tmp_path / f"rank{r}.npz") for r in (0, 1))
    for z in (r0, r1):
        assert np.array_equal(z["positions"], np.stack([np.asarray(r.positions) for r in recs]))
        np.testing.assert_allclose(z["losses"], [r.loss for r in recs], rtol=1e-5)
        for k, v in ref.online.items():
            np.testing.assert_allclose(z["on_" + k], v.numpy(), atol=1e-5, rtol=0, err_msg=k)
            np.testing.assert_allclose(z["tg_" + k], ref.target[k].numpy(), atol=1e-5, rtol=0, err_msg=k)
        if ref.per:
            np.testing.assert_allclose(z["tree"], ref.replay.replay_buffer.tree, rtol=1e-6, atol=1e-6)
    for k in ref.online:   # replicas stay bitwise identical across ranks
        assert np.array_equal(r0["on_" + k], r1["on_" + k])


class BucketedOracleShardEngine(OracleShardEngine):
    """The bucket surface of LearnEngine (dp_buckets / learn_step_bucket / apply_grads_bucket)
    over the oracle shard: bucket b's gradient range is published only by learn_step_bucket(b),
    so an all-reduce that ran early, twice or over the wrong range changes the result; the full
    update is applied when the last bucket's apply arrives.  The call order is logged."""

    def __init__(self, learner, world, rank):
        super().__init__(learner, world, rank)
        sizes = [v.numel() for v in learner.online.values()]
        # reverse layer order, like the engine: the last tensors (head) + the loss slot first
        cut1 = self.P - sum(sizes[-2:])
        cut2 = sizes[0] + sizes[1]
        self.buckets = [(cut1, self.P - cut1 + 1), (cut2, cut1 - cut2), (0, cut2)]
        self.full = None
        self.log = []

    def dp_buckets(self):
        return list(self.buckets)

    def learn_step_bucket(self, b):
        self.log.append(("learn", b))
        if b == 0:
            self.grads.zero_()
            self.learn_step(grads_only=True)
            self.full = self.grads.clone()
            self.grads.zero_()
        f, c = self.buckets[b]
        self.grads[f:f + c] = self.full[f:f + c]

    def apply_grads_bucket(self, b, soft_update=True):
        self.log.append(("apply", b))
        if b == len(self.buckets) - 1:
            self.apply_grads(soft_update=soft_update)


def bucket_worker(rank, world, port, algo, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from dqn.data_parallel import dp_learn_step, dp_learn_step_bucketed
    plain = OracleShardEngine(make_learner(algo), world, rank)
    buck = BucketedOracleShardEngine(make_learner(algo), world, rank)
    for _ in range(3):
        dp_learn_step(plain, soft_update=True)
        dp_learn_step_bucketed(buck, soft_update=True)
    np.savez(os.path.join(out_dir, f"b{rank}.npz"),
             plain=torch.cat([v.reshape(-1) for v in plain.L.online.values()]).numpy(),
             buck=torch.cat([v.reshape(-1) for v in buck.L.online.values()]).numpy(),
             plain_t=torch.cat([v.reshape(-1) for v in plain.L.target.values()]).numpy(),
             buck_t=torch.cat([v.reshape(-1) for v in buck.L.target.values()]).numpy(),
             log=np.array([[0 if k == "learn" else 1, b] for k, b in buck.log]))
    dist.destroy_process_group()


@pytest.mark.parametrize("algo", ALGOS)
def test_bucketed_dp_step_order_and_identity(tmp_path, algo):
    """dqn.data_parallel.dp_learn_step_bucketed on 2 gloo ranks: buckets are completed, all-reduced
    and applied in order 0, 1, 2 (learn_step_bucket(b) before apply_grads_bucket(b), before
    learn_step_bucket(b+1)), and the result equals the single all-reduce step exactly."""
    port = free_port()
    mp.spawn(bucket_worker, args=(2, port, algo, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        z = np.load(tmp_path / f"b{r}.npz")
        assert np.array_equal(z["plain"], z["buck"]) and np.array_equal(z["plain_t"], z["buck_t"])
        want = [[k, b] for _ in range(3) for b in range(3) for k in (0, 1)]
        assert z["log"].tolist() == want
