"""MI355X-native drop-in for the reference's ``dqn`` package hot path
(dqn.agent / dqn.network / dqn.replay_memory of youcefMehamlia/Multimodal-DRL-RMC).

    import sys; sys.path.insert(0, ".../multimodal-drl-rmc_amd")
    from dqn import Agents, Networks     # same names as R:dqn/__init__.py:3-4

The learn step runs in libdqnx.so (hand-written gfx950 HIP kernels); see DESIGN.md.
The env wrappers the reference's package also exports (CustomEnvWrapper, make_env) belong
to the SUMO loop, which stays with the reference.
"""
from . import engine  # noqa: F401
from . import network as Networks  # noqa: F401
from . import agent as Agents  # noqa: F401

__all__ = ["Agents", "Networks", "engine"]
