"""MI355X-native drop-in for the reference's ``dqn`` package hot path
(dqn.agent / dqn.network / dqn.replay_memory of youcefMehamlia/Multimodal-DRL-RMC).

    import sys; sys.path.insert(0, ".../multimodal-drl-rmc_amd")
    from dqn import Agents        # same name as R:dqn/__init__.py:3

The learn step runs in libdqnx.so (hand-written gfx950 HIP kernels); see DESIGN.md.
"""
from . import engine  # noqa: F401
