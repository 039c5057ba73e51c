"""GPU: the drop-in agents driven like R:train.py's loop (choose_actions -> store_transitions
-> learn -> update_target_network), against the oracle learner on the same seeds.  Checks
the global RNG hand-off (Python random for uniform replay, numpy for PER) as well as the
weights."""
import random

import numpy as np
import pytest
import torch

from dqn import Agents
from dqn import _capi as C
from oracle import ref as O
from refnets import agent_kwargs, hybrid_network_config, mse_network_config, rmsprop_network_config

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("algo,obs_dim,batch,buffer,n_fill,net,n_env", [
    ("DQNAgent", 14, 32, 500, 300, "mlp", 1),
    ("DuelingDoubleDQNAgent", 284, 64, 1000, 700, "mlp", 1),
    ("PerDuelingDoubleDQNAgent", 284, 64, 1000, 700, "mlp", 1),
    # the reference's HEAD configuration: DuelingDoubleDQNAgent on env/dqn_config.network_config
    # (TwoStreamHybridNetwork), as bin/train.sh launches it (R:train.py:24, R:bin/train.sh:5)
    ("DuelingDoubleDQNAgent", 284, 64, 1000, 700, "hybrid", 1),
    ("PerDuelingDoubleDQNAgent", 284, 32, 500, 300, "hybrid", 1),
    # -n_env 2 (R:train.py:120): two rows per store_transitions / choose_actions, soft update with
    # tau*n_env (R:dqn/agent.py:105-110), PER beta at step*n_env (R:dqn/agent.py:247); a ring
    # that wraps during the loop (uniform) and a buffer filled to capacity (PER)
    ("DuelingDoubleDQNAgent", 284, 64, 706, 700, "mlp", 2),
    ("PerDuelingDoubleDQNAgent", 284, 64, 700, 700, "mlp", 2),
    ("DQNAgent", 14, 32, 500, 300, "mlp", 3),
    ("PerDuelingDoubleDQNAgent", 284, 32, 500, 300, "hybrid", 2),
])
def test_gpu_agent_train_loop_matches_oracle(tmp_path, algo, obs_dim, batch, buffer, n_fill, net, n_env):
    seed = 17
    torch.manual_seed(seed)
    over = {"nn_conf_func": hybrid_network_config} if net == "hybrid" else {}
    agent = getattr(Agents, algo)(**agent_kwargs(algo, obs_dim, batch, buffer, tmp_path, n_env=n_env, **over))
    head = O.algo_spec_head(algo)
    spec = O.hybrid_spec(8, head) if net == "hybrid" else O.mlp_spec(obs_dim, 8, head)
    init = O.reference_init(spec, seed)
    for k, v in agent.online_network.state_dict().items():
        assert torch.equal(v.cpu(), init[k]), k
    oracle = O.OracleLearner(spec, algo, batch, buffer, seed=seed, params=init, per_pow="cr", n_env=n_env)

    steps = 4
    obs, act, rew, done, nobs = O.synth_transitions(n_fill + steps * n_env, obs_dim, 8, seed=seed)
    for i in range(0, n_fill, n_env):   # init_replay_memory_buffer: n_env rows per env step (R:train.py:63-81)
        j = min(i + n_env, n_fill)
        rows = (obs[i:j], [int(a) for a in act[i:j]], [float(r) for r in rew[i:j]], [bool(d) for d in done[i:j]],
                nobs[i:j])
        agent.store_transitions(*rows, None)
        oracle.store_transitions(*rows)

    random.seed(seed)
    np.random.seed(seed)
    for t in range(steps):
        agent.step = t
        agent.epsilon_start = 0.5          # mix greedy and random actions
        lo, hi = n_fill + t * n_env, n_fill + (t + 1) * n_env
        x = obs[lo:hi]
        s0 = random.getstate()
        actions = agent.choose_actions(x)
        s1 = random.getstate()
        # oracle acting: same draws on the same stream (R:dqn/agent.py:92-99)
        random.setstate(s0)
        ref_actions = O.greedy_actions(spec, oracle.online, x)
        for i in range(len(ref_actions)):
            if random.random() <= agent.epsilon():
                ref_actions[i] = random.randint(0, 7)
        assert random.getstate() == s1 and actions == ref_actions
        if n_env > 1:   # the env step's n_env transitions reach the replay before learn() (R:train.py:93-99)
            rows = (x, list(actions), [float(r) for r in rew[lo:hi]], [bool(d) for d in done[lo:hi]], nobs[lo:hi])
            agent.store_transitions(*rows, None)
            oracle.store_transitions(*rows)

        oracle.py_state = O.py_state_to_array()
        oracle.np_state = O.np_state_to_array()
        oracle.step = t
        agent.learn()
        agent.update_target_network()
        rec = oracle.learn()
        oracle.update_target_network()
        # no flush: learn() leaves the global generators where the reference's draw leaves them
        assert np.array_equal(np.asarray(random.getstate()[1], dtype=np.uint32), oracle.py_state)
        assert np.array_equal(O.np_state_to_array(), oracle.np_state)
        assert abs(agent.engine.loss() - rec.loss) <= 1e-5 * max(1.0, abs(rec.loss))
        on, tg = agent.online_network.state_dict(), agent.target_network.state_dict()
        for k in init:
            np.testing.assert_allclose(on[k].cpu().numpy(), oracle.online[k].numpy(), atol=1e-5, rtol=0, err_msg=k)
            np.testing.assert_allclose(tg[k].cpu().numpy(), oracle.target[k].numpy(), atol=1e-5, rtol=0, err_msg=k)

    # checkpoint written from engine memory reloads into a fresh network
    p = str(tmp_path / "ck.pack")
    agent.step = 5
    agent.online_network.save(p, 5, 0, 0.0, 0.0)
    agent.online_network.load(p)
    for k in init:
        np.testing.assert_allclose(agent.online_network.state_dict()[k].cpu().numpy(),
                                   oracle.online[k].numpy(), atol=1e-5, rtol=0)


@pytest.mark.parametrize("conf", [rmsprop_network_config, mse_network_config])
def test_gpu_agent_refuses_other_optimizer_or_loss(tmp_path, conf):
    """network_config may name RMSprop / MSELoss; the engine implements Adam + SmoothL1 only and
    must refuse instead of training with a different update rule."""
    with pytest.raises(NotImplementedError):
        Agents.DuelingDoubleDQNAgent(**agent_kwargs("DuelingDoubleDQNAgent", 14, 32, 500, tmp_path,
                                                    nn_conf_func=conf))


def test_gpu_agent_log_reports_learn_throughput(tmp_path):
    """Agent.log adds the learn-throughput scalar (transitions/s) next to the reference's
    AvgRew / AvgEpLen / Episodes (R:dqn/agent.py:130-147)."""
    agent = Agents.DuelingDoubleDQNAgent(**agent_kwargs("DuelingDoubleDQNAgent", 14, 32, 500, tmp_path,
                                                        log_frequency=2))
    obs, act, rew, done, nobs = O.synth_transitions(100, 14, 8, seed=1)
    for i in range(100):
        agent.store_transitions(obs[i:i + 1], [int(act[i])], [float(rew[i])], [bool(done[i])], nobs[i:i + 1], None)
    seen = {}
    agent.summary_writer.add_scalar = lambda tag, v, global_step=None: seen.__setitem__(tag, v)
    for t in range(3):
        agent.step = t
        agent.learn()
        agent.update_target_network()
        agent.log()
    assert {"AvgRew", "AvgEpLen", "Episodes", "Loss", "LearnTransitionsPerSec"} <= set(seen)
    assert seen["LearnTransitionsPerSec"] > 0


def test_gpu_per_agent_step_survives_host_sampling(tmp_path):
    """A host-side ReplayMemoryPrioritized.sample_transitions(step) moves the engine's PER step;
    the next learn() must still interpolate beta from agent.step (ADVICE: stale cached step)."""
    agent = Agents.PerDuelingDoubleDQNAgent(**agent_kwargs("PerDuelingDoubleDQNAgent", 14, 32, 500, tmp_path))
    obs, act, rew, done, nobs = O.synth_transitions(100, 14, 8, seed=2)
    for i in range(100):
        agent.store_transitions(obs[i:i + 1], [int(act[i])], [float(rew[i])], [bool(done[i])], nobs[i:i + 1], None)
    agent.step = 7
    agent.learn()
    agent.replay_memory_buffer.sample_transitions(123456)
    agent.step = 8
    agent.learn()
    torch.cuda.synchronize()
    beta = float(agent.engine.ctrl().per_beta)
    assert abs(beta - float(np.interp(8, [0, 2e6], [0.4, 1.0]))) < 1e-12, beta


def test_gpu_agent_drives_gymnasium_env_through_adapter(tmp_path):
    """R:train.py's init_replay_memory_buffer + train_loop over dqn.env_adapter.GymnasiumVecEnv
    (gymnasium 5-tuple envs): the replay ring holds exactly the transitions the
    env produced (reset observations in new_obs at episode ends, as DummyVecEnv stores them), and
    finished episodes reach the agent's episode buffer."""
    from dqn.env_adapter import GymnasiumVecEnv
    from test_env_adapter import ToyEnv

    class Env284(ToyEnv):
        def __init__(self):
            super().__init__(length=5, dim=14)

    env = GymnasiumVecEnv([Env284])
    agent = Agents.DuelingDoubleDQNAgent(**agent_kwargs("DuelingDoubleDQNAgent", 14, 8, 100, tmp_path))
    seen = []
    obses = env.reset()
    for t in range(12):                                # init_replay_memory_buffer (R:train.py:63-81)
        actions = [t % 8]
        new_obses, rews, dones, infos = env.step(actions)
        agent.store_transitions(obses, actions, rews, dones, new_obses, infos)
        seen.append((obses[0].copy(), actions[0], float(rews[0]), bool(dones[0]), new_obses[0].copy()))
        obses = new_obses
    for step in range(3):                              # train_loop (R:train.py:83-108)
        agent.step = step
        actions = agent.choose_actions(obses)
        new_obses, rews, dones, infos = env.step(actions)
        agent.store_transitions(obses, actions, rews, dones, new_obses, infos)
        seen.append((obses[0].copy(), int(actions[0]), float(rews[0]), bool(dones[0]), new_obses[0].copy()))
        obses = new_obses
        agent.learn()
        agent.update_target_network()
    ring = agent.replay_memory_buffer.replay_buffer
    assert len(ring) == len(seen)
    for i, (o, a, r, d, no) in enumerate(seen):
        ro, ra, rr, rd, rno = ring[i]
        assert np.array_equal(ro, o) and ra == a and rr == np.float32(r) and rd == d and np.array_equal(rno, no), i
    assert agent.episode_count == sum(1 for s in seen if s[3])


@pytest.mark.parametrize("algo,soft", [("DuelingDoubleDQNAgent", True), ("DuelingDoubleDQNAgent", False),
                                       ("PerDuelingDoubleDQNAgent", True), ("DQNAgent", True)])
def test_gpu_agent_deferred_learn_bit_identical(tmp_path, monkeypatch, algo, soft):
    """learn() records the step and the next agent call launches it (update_target_network with the
    soft update fused into the Adam pass; RNG hand-back through pinned buffers, installed lazily):
    bitwise the synchronous learn() (DQNX_AGENT_DEFER=0) over a train.py loop, hard target updates
    (every 3 steps) included, the global RNG states after every iteration and the logged loss; and the
    in-place staging of random._inst (dqnx_agent_learn_mt) bitwise the portable getstate / getrandbits
    hand-off (DQNX_AGENT_MT_INPLACE=0)."""
    runs = []
    # (+ the portable getstate / getrandbits hand-off, and the RNG upload copy instead of the sampler
    #  reading the pinned block in place)
    for defer, inplace, zc in (("0", "1", "1"), ("1", "1", "1"), ("0", "0", "1"), ("0", "1", "0")):
        monkeypatch.setenv("DQNX_AGENT_DEFER", defer)
        monkeypatch.setenv("DQNX_AGENT_MT_INPLACE", inplace)
        monkeypatch.setenv("DQNX_AGENT_ZC", zc)
        torch.manual_seed(5)
        agent = getattr(Agents, algo)(**agent_kwargs(algo, 284, 64, 1000, tmp_path, target_soft_update=soft,
                                                     update_target_frequency=3))
        obs, act, rew, done, nobs = O.synth_transitions(800, 284, 8, seed=9)
        for i in range(700):
            agent.store_transitions(obs[i:i + 1], [int(act[i])], [float(rew[i])], [bool(done[i])], nobs[i:i + 1],
                                    None)
        random.seed(3)
        np.random.seed(3)
        states = []
        for t in range(8):
            agent.step = t
            agent.epsilon_start = 0.5
            a = agent.choose_actions(obs[700 + t:701 + t])
            agent.store_transitions(obs[700 + t:701 + t], a, [float(rew[700 + t])], [False], nobs[700 + t:701 + t], None)
            agent.learn()
            agent.update_target_network()
            states.append((a, random.getstate()))
        agent.flush()
        torch.cuda.synchronize()
        runs.append((agent, states, random.getstate(), np.random.get_state()[1].copy(), agent.engine.loss()))
    a0, s0, r0, n0, l0 = runs[0]
    for a1, s1, r1, n1, l1 in runs[1:]:
        assert s0 == s1   # actions and the global state after every iteration
        assert r0 == r1 and np.array_equal(n0, n1) and l0 == l1
        assert torch.equal(a0.engine.params, a1.engine.params)
        assert torch.equal(a0.engine.target_params, a1.engine.target_params)
        assert torch.equal(a0.engine.adam_m, a1.engine.adam_m)


@pytest.mark.parametrize("algo,net", [("DuelingDoubleDQNAgent", "mlp"), ("PerDuelingDoubleDQNAgent", "mlp"),
                                      ("DQNAgent", "mlp"), ("DuelingDoubleDQNAgent", "hybrid")])
def test_gpu_agent_reads_after_learn_see_the_step(tmp_path, algo, net):
    """R:dqn/agent.py:204-226 is synchronous: right after learn() (no update_target_network, no flush)
    the online network's forward / value / advantages and parameters() read the post-step weights, and
    the global RNG has moved past the step's draw."""
    seed = 23
    torch.manual_seed(seed)
    over = {"nn_conf_func": hybrid_network_config} if net == "hybrid" else {}
    agent = getattr(Agents, algo)(**agent_kwargs(algo, 284, 64, 1000, tmp_path, **over))
    head = O.algo_spec_head(algo)
    spec = O.hybrid_spec(8, head) if net == "hybrid" else O.mlp_spec(284, 8, head)
    init = O.reference_init(spec, seed)
    oracle = O.OracleLearner(spec, algo, 64, 1000, seed=seed, params=init, per_pow="cr")
    obs, act, rew, done, nobs = O.synth_transitions(700, 284, 8, seed=seed)
    rows = (obs, [int(a) for a in act], [float(r) for r in rew], [bool(d) for d in done], nobs)
    agent.store_transitions(*rows, None)
    oracle.store_transitions(*rows)
    random.seed(seed)
    np.random.seed(seed)
    x = torch.as_tensor(obs[:16], device=agent.device)
    for t in range(2):
        agent.step = oracle.step = t
        oracle.py_state = O.py_state_to_array()
        oracle.np_state = O.np_state_to_array()
        agent.learn()
        oracle.learn()
        assert np.array_equal(np.asarray(random.getstate()[1], dtype=np.uint32), oracle.py_state)
        assert np.array_equal(O.np_state_to_array(), oracle.np_state)
        with torch.no_grad():
            q = agent.online_network(x).cpu()
        q_ref = O.q_forward(spec, oracle.online, x.cpu())
        np.testing.assert_allclose(q.numpy(), q_ref.numpy(), atol=1e-5, rtol=0)
        if head == "dueling":
            with torch.no_grad():
                adv = agent.online_network.advantages(x).cpu()
            np.testing.assert_allclose(adv.numpy(), O.advantages(spec, oracle.online, x.cpu()).numpy(), atol=1e-5)
        agent.update_target_network()
        oracle.update_target_network()
    got = {k: p.detach().cpu() for k, p in agent.online_network.named_parameters()}
    for k in init:
        np.testing.assert_allclose(got[k].numpy(), oracle.online[k].numpy(), atol=1e-5, rtol=0, err_msg=k)


def test_gpu_agent_learn_raises_on_short_replay(tmp_path):
    """random.sample(deque, batch_size) raises ValueError when fewer transitions are stored
    (R:dqn/replay_memory.py:39): learn() on a 10-row buffer with batch 32 does too, leaves the global
    RNG untouched, and the agent keeps working once the buffer holds enough."""
    agent = Agents.DuelingDoubleDQNAgent(**agent_kwargs("DuelingDoubleDQNAgent", 14, 32, 500, tmp_path))
    obs, act, rew, done, nobs = O.synth_transitions(40, 14, 8, seed=3)
    agent.store_transitions(obs[:10], [int(a) for a in act[:10]], [float(r) for r in rew[:10]],
                            [bool(d) for d in done[:10]], nobs[:10], None)
    s0 = random.getstate()
    with pytest.raises(ValueError, match="Sample larger than population"):
        agent.learn()
    assert random.getstate() == s0
    agent.store_transitions(obs[10:], [int(a) for a in act[10:]], [float(r) for r in rew[10:]],
                            [bool(d) for d in done[10:]], nobs[10:], None)
    agent.learn()
    agent.update_target_network()
    agent.choose_actions(obs[:1])


def test_gpu_agent_surfaces_device_errors(tmp_path):
    """A sticky device error (dqnx_ctrl.error, e.g. the PER tree hand-off timing out inside a launch)
    comes back with the control block after the step and is raised at the agent's next
    synchronisation point instead of training on silently."""
    agent = Agents.PerDuelingDoubleDQNAgent(**agent_kwargs("PerDuelingDoubleDQNAgent", 14, 32, 500, tmp_path))
    obs, act, rew, done, nobs = O.synth_transitions(100, 14, 8, seed=4)
    agent.store_transitions(obs, [int(a) for a in act], [float(r) for r in rew], [bool(d) for d in done], nobs, None)
    agent.learn()
    agent.update_target_network()
    agent.choose_actions(obs[:1])   # clean so far
    err_off = C.Ctrl.error.offset
    agent.engine.ctrl_bytes[err_off:err_off + 4].view(torch.int32).fill_(C.DEVERR_PER_HANDOFF)
    agent.learn()
    agent.update_target_network()
    with pytest.raises(RuntimeError, match="hand-off"):
        agent.choose_actions(obs[:1])
