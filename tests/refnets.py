"""Test helpers: the reference's network_config shapes (restated, R:env/custom_env/macro with
lane/dqn_config.py:58-104) and a gym-Box stand-in for `input_dim`."""
import torch.nn as nn
import torch.optim as optim


class Box:
    def __init__(self, n):
        self.shape = (n,)


def mlp_network_config(input_dim_space):
    n = input_dim_space.shape[0]
    act = nn.ReLU()                       # one shared instance, like the reference
    net = nn.Sequential(nn.Linear(n, 256), act, nn.Linear(256, 128), act)
    return net, 128, optim.Adam, nn.SmoothL1Loss


def agent_kwargs(algo, obs_dim, batch, buffer, tmpdir, **over):
    kw = dict(n_env=1, lr=1e-4, gamma=0.99, epsilon_start=1.0, epsilon_min=0.05, epsilon_decay=2e6,
              epsilon_exp_decay=False, nn_conf_func=mlp_network_config, input_dim=Box(obs_dim), output_dim=8,
              batch_size=batch, min_buffer_size=batch, buffer_size=buffer, update_target_frequency=30000,
              target_soft_update=True, target_soft_update_tau=1e-3, save_frequency=1000, log_frequency=1000,
              save_dir=str(tmpdir) + "/", log_dir=str(tmpdir) + "/", load=False, algo=algo, gpu="0")
    kw.update(over)
    return kw
