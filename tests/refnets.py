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


class TwoStreamHybridNetwork(nn.Module):
    """The reference's HEAD Q-network body restated for the tests (R:env/dqn_config.py:66-143),
    with its attribute names (macro_len, micro_shape, cnn_stream, dense_stream, fc_out_dim):
    [Conv2d(k, stride, padding k//2), act]* over the (c,h,w) micro grid viewed from x[:, macro_len:],
    flatten ++ macro, then [Linear, act]*."""

    def __init__(self, macro_vec_len, micro_shape_chw, cnn_params, dense_params, activation_fn):
        super().__init__()
        self.macro_len = macro_vec_len
        self.micro_shape = micro_shape_chw
        layers, c = [], micro_shape_chw[0]
        h, w = micro_shape_chw[1], micro_shape_chw[2]
        for filters, kernel, stride in cnn_params:
            layers += [nn.Conv2d(c, filters, kernel_size=kernel, stride=stride,
                                 padding=(kernel[0] // 2, kernel[1] // 2)), activation_fn]
            h = (h + 2 * (kernel[0] // 2) - kernel[0]) // stride[0] + 1
            w = (w + 2 * (kernel[1] // 2) - kernel[1]) // stride[1] + 1
            c = filters
        self.cnn_stream = nn.Sequential(*layers)
        dense, d = [], c * h * w + macro_vec_len
        for out in dense_params:
            dense += [nn.Linear(d, out), activation_fn]
            d = out
        self.dense_stream = nn.Sequential(*dense)
        self.fc_out_dim = d

    def forward(self, x):
        import torch
        macro = x[:, :self.macro_len]
        micro = x[:, self.macro_len:].view(-1, *self.micro_shape)
        feat = self.cnn_stream(micro).flatten(start_dim=1)
        return self.dense_stream(torch.cat([feat, macro], dim=1))


def hybrid_network_config(input_dim_space, micro_chw=(2, 27, 5)):
    """network_config of R:env/dqn_config.py:148-193 (ELU, Adam, SmoothL1)."""
    net = TwoStreamHybridNetwork(14, micro_chw, [(32, (3, 3), (1, 1)), (64, (3, 3), (2, 1)), (64, (3, 3), (2, 2))],
                                 [512, 256], nn.ELU())
    return net, net.fc_out_dim, optim.Adam, nn.SmoothL1Loss


def rmsprop_network_config(input_dim_space):
    """An MLP config that names RMSprop (R:env/custom_env/macro with lane/dqn_config.py:96)."""
    net, out, _, loss = mlp_network_config(input_dim_space)
    return net, out, optim.RMSprop, loss


def mse_network_config(input_dim_space):
    """An MLP config that names MSELoss (R:env/custom_env/macro with lane/dqn_config.py:101)."""
    net, out, opt, _ = mlp_network_config(input_dim_space)
    return net, out, opt, nn.MSELoss
