"""GPU: the drop-in agents driven like R:train.py's loop (choose_actions -> store_transitions
-> learn -> update_target_network), against the oracle learner on the same seeds.  Checks
the global RNG hand-off (Python random for uniform replay, numpy for PER) as well as the
weights."""
import random

import numpy as np
import pytest
import torch

from dqn import Agents
from oracle import ref as O
from refnets import agent_kwargs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("algo,obs_dim,batch,buffer,n_fill", [
    ("DQNAgent", 14, 32, 500, 300),
    ("DuelingDoubleDQNAgent", 284, 64, 1000, 700),
    ("PerDuelingDoubleDQNAgent", 284, 64, 1000, 700),
])
def test_gpu_agent_train_loop_matches_oracle(tmp_path, algo, obs_dim, batch, buffer, n_fill):
    seed = 17
    torch.manual_seed(seed)
    agent = getattr(Agents, algo)(**agent_kwargs(algo, obs_dim, batch, buffer, tmp_path))
    head = O.algo_spec_head(algo)
    spec = O.mlp_spec(obs_dim, 8, head)
    init = O.reference_init(spec, seed)
    for k, v in agent.online_network.state_dict().items():
        assert torch.equal(v.cpu(), init[k]), k
    oracle = O.OracleLearner(spec, algo, batch, buffer, seed=seed, params=init, per_pow="cr")

    obs, act, rew, done, nobs = O.synth_transitions(n_fill + 8, obs_dim, 8, seed=seed)
    for i in range(n_fill):   # init_replay_memory_buffer: one env step (n_env = 1) at a time
        agent.store_transitions(obs[i:i + 1], [int(act[i])], [float(rew[i])], [bool(done[i])], nobs[i:i + 1], None)
    O.fill_replay(oracle, obs[:n_fill], act[:n_fill], rew[:n_fill], done[:n_fill], nobs[:n_fill])

    random.seed(seed)
    np.random.seed(seed)
    for t in range(4):
        agent.step = t
        agent.epsilon_start = 0.5          # mix greedy and random actions
        x = obs[n_fill + t:n_fill + t + 1]
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

        oracle.py_state = O.py_state_to_array()
        oracle.np_state = O.np_state_to_array()
        oracle.step = t
        agent.learn()
        agent.update_target_network()
        rec = oracle.learn()
        oracle.update_target_network()
        torch.cuda.synchronize()
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
