"""``jax.numpy`` subset used by the case studies (``case4_gspmd_ff.py:30``, ``case6_attention.py:110-135``)."""
from __future__ import annotations

import numpy as _np
import torch as _torch

from . import dtypes as _dt
from .array import ShardedArray, device_put as _device_put
from .ops import core as _core

float32 = _dt.float32
float16 = _dt.float16
bfloat16 = _dt.bfloat16
int32 = _dt.int32
int8 = _dt.int8
float8_e4m3fn = _dt.float8_e4m3fn
float8_e5m2 = _dt.float8_e5m2
dtype = _dt.canonicalize
ndarray = ShardedArray


def asarray(x, dtype=None):
    if isinstance(x, ShardedArray):
        return x if dtype is None else _core.convert(x, dtype)
    a = _device_put(_np.asarray(x))
    return a if dtype is None else _core.convert(a, dtype)


array = asarray


def _mk(name, dt):
    def conv(x):
        return asarray(x, dt)
    conv.__name__ = name
    return conv


# ``jnp.float32(q)`` casts (case6_attention.py:121-122)
globals()["float32"] = type("float32", (), {"__new__": lambda cls, x=0.0: asarray(x, _torch.float32),
                                            "dtype": _torch.float32})
globals()["bfloat16"] = type("bfloat16", (), {"__new__": lambda cls, x=0.0: asarray(x, _torch.bfloat16),
                                              "dtype": _torch.bfloat16})
globals()["float16"] = type("float16", (), {"__new__": lambda cls, x=0.0: asarray(x, _torch.float16),
                                            "dtype": _torch.float16})

einsum = _core.einsum
matmul = _core.matmul
dot = _core.dot
reshape = lambda a, newshape: _core.reshape(a, newshape)  # noqa: E731
transpose = lambda a, axes=None: _core.transpose(a, axes if axes is not None else tuple(reversed(range(a.ndim))))  # noqa: E731
sum = lambda a, axis=None, keepdims=False, dtype=None: _core.reduce_sum(a, axis, keepdims, dtype)  # noqa: E731,A001
mean = lambda a, axis=None, keepdims=False: _core.reduce_mean(a, axis, keepdims)  # noqa: E731
max = lambda a, axis=None, keepdims=False: _core.reduce_max(a, axis, keepdims)  # noqa: E731,A001
exp = lambda a: _core.unary("exp", a)  # noqa: E731
log = lambda a: _core.unary("log", a)  # noqa: E731
tanh = lambda a: _core.unary("tanh", a)  # noqa: E731
sqrt = lambda a: _core.unary("sqrt", a)  # noqa: E731
maximum = lambda a, b: _core.binary("max", a, b)  # noqa: E731
minimum = lambda a, b: _core.binary("min", a, b)  # noqa: E731
where = _core.where
concatenate = lambda arrs, axis=0: _core.concatenate(arrs, axis)  # noqa: E731
broadcast_to = _core.broadcast_to
array_equal = lambda a, b: bool(_np.array_equal(_np.asarray(a), _np.asarray(b)))  # noqa: E731
allclose = lambda a, b, rtol=1e-5, atol=1e-8: bool(_np.allclose(_np.asarray(a), _np.asarray(b), rtol, atol))  # noqa: E731


def zeros(shape, dtype=None, device=None):
    return _device_put(_torch.zeros(shape, dtype=_dt.canonicalize(dtype) or _torch.float32), device)


def ones(shape, dtype=None, device=None):
    return _device_put(_torch.ones(shape, dtype=_dt.canonicalize(dtype) or _torch.float32), device)


def arange(start, stop=None, step=None, dtype=None):
    """``jnp.arange``: int32 for integer arguments, float32 if any is a float (JAX's defaults)."""
    args = [a for a in (start, stop, step) if a is not None]
    if dtype is None:
        dtype = _torch.float32 if any(isinstance(a, float) for a in args) else _torch.int32
    if stop is None:
        start, stop = 0, start
    return _device_put(_torch.arange(start, stop, 1 if step is None else step, dtype=_dt.canonicalize(dtype) or dtype))
