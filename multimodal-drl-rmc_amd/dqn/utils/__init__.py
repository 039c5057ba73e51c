"""Helpers of the drop-in `dqn` package: the `.pack` checkpoint codec."""
from .pack import dumps, loads, save_pack, load_pack

__all__ = ["dumps", "loads", "save_pack", "load_pack"]
