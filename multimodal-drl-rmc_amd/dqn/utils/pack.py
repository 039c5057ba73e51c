"""`.pack` checkpoints: msgpack with numpy values, wire-compatible with the reference's
`Network.save` / `Network.load` (R:dqn/network.py:27-47), which serialise through the
msgpack-numpy extension hooks (R:dqn/utils/msgpack_numpy.py:74-143).

Wire format of a numpy value (msgpack map with bytes keys):
  array:  {b'nd': True,  b'type': dtype.str, b'kind': b'', b'shape': [...], b'data': raw bytes}
  scalar: {b'nd': False, b'type': dtype.str, b'data': raw bytes}
Only plain dtypes are supported (structured dtypes never occur in Q-network checkpoints).
Decoding never executes anything from the file: numpy arrays are rebuilt with frombuffer.
"""
from __future__ import annotations

import os

import msgpack
import numpy as np


def _default(obj):
    if isinstance(obj, np.ndarray):
        if obj.dtype.kind == "V":
            raise TypeError("structured dtypes are not supported in .pack checkpoints")
        return {b"nd": True, b"type": obj.dtype.str, b"kind": b"", b"shape": list(obj.shape),
                b"data": np.ascontiguousarray(obj).tobytes()}
    if isinstance(obj, (np.bool_, np.number)):
        return {b"nd": False, b"type": obj.dtype.str, b"data": obj.tobytes()}
    raise TypeError(f"cannot serialise {type(obj).__name__}")


def _hook(obj):
    nd = obj.get(b"nd")
    if nd is True:
        if obj.get(b"kind") == b"V":
            raise ValueError("structured dtypes are not supported in .pack checkpoints")
        dt = np.dtype(obj[b"type"])
        return np.frombuffer(obj[b"data"], dtype=dt).reshape(obj[b"shape"]).copy()
    if nd is False:
        return np.frombuffer(obj[b"data"], dtype=np.dtype(obj[b"type"]))[0]
    return obj


def dumps(obj) -> bytes:
    return msgpack.packb(obj, default=_default, use_bin_type=True)


def loads(data: bytes):
    return msgpack.unpackb(data, object_hook=_hook, raw=False, strict_map_key=False)


def save_pack(path: str, parameters: dict, step, episode_count, rew_mean, len_mean):
    """Network.save layout (R:dqn/network.py:27-35)."""
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    blob = dumps({"parameters": parameters, "step": step, "episode_count": episode_count,
                  "rew_mean": rew_mean, "len_mean": len_mean})
    with open(path, "wb") as f:
        f.write(blob)


def load_pack(path: str):
    """-> (parameters dict name -> ndarray, step, episode_count, rew_mean, len_mean)
    (R:dqn/network.py:37-47)."""
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    with open(path, "rb") as f:
        d = loads(f.read())
    return d["parameters"], d["step"], d["episode_count"], d["rew_mean"], d["len_mean"]
