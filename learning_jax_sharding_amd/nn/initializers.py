"""Parameter initializers (``flax.linen.initializers`` subset).

``lecun_normal`` (``case6_attention.py:57``): variance scaling, fan_in mode,
truncated normal on [-2, 2] with the 0.87962566 correction, drawn with the
shard-invariant Philox generator so each device creates only its shard.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import numpy as np
import torch

from .. import dtypes as _dt
from .. import random as _random

__all__ = ["lecun_normal", "zeros", "ones", "normal", "variance_scaling", "xavier_uniform", "zeros_init",
           "glorot_normal", "he_normal", "constant"]


def _fans(shape: Sequence[int], in_axis=-2, out_axis=-1):
    shape = tuple(shape)
    if len(shape) < 1:
        return 1, 1
    if len(shape) == 1:
        return shape[0], shape[0]
    rf = int(np.prod([s for i, s in enumerate(shape) if i not in (in_axis % len(shape), out_axis % len(shape))]))
    return shape[in_axis] * rf, shape[out_axis] * rf


def variance_scaling(scale: float, mode: str, distribution: str, in_axis=-2, out_axis=-1, dtype=None):
    def init(key, shape, dtype_=None, sharding=None):
        dt = _dt.canonicalize(dtype_ or dtype) or torch.float32
        fan_in, fan_out = _fans(shape, in_axis, out_axis)
        denom = {"fan_in": fan_in, "fan_out": fan_out, "fan_avg": (fan_in + fan_out) / 2}[mode]
        var = scale / max(1.0, denom)
        if distribution == "truncated_normal":
            std = math.sqrt(var) / 0.87962566103423978
            return _random.truncated_normal(key, -2.0, 2.0, shape, dt, sharding=sharding) * std
        if distribution == "normal":
            return _random.normal(key, shape, dt, sharding=sharding) * math.sqrt(var)
        if distribution == "uniform":
            lim = math.sqrt(3 * var)
            return _random.uniform(key, shape, dt, -lim, lim, sharding=sharding)
        raise ValueError(distribution)
    return init


def lecun_normal(in_axis=-2, out_axis=-1, dtype=None):
    return variance_scaling(1.0, "fan_in", "truncated_normal", in_axis, out_axis, dtype)


def glorot_normal(in_axis=-2, out_axis=-1, dtype=None):
    return variance_scaling(1.0, "fan_avg", "truncated_normal", in_axis, out_axis, dtype)


def he_normal(in_axis=-2, out_axis=-1, dtype=None):
    return variance_scaling(2.0, "fan_in", "truncated_normal", in_axis, out_axis, dtype)


def xavier_uniform(in_axis=-2, out_axis=-1, dtype=None):
    return variance_scaling(1.0, "fan_avg", "uniform", in_axis, out_axis, dtype)


def normal(stddev: float = 1e-2, dtype=None):
    def init(key, shape, dtype_=None, sharding=None):
        return _random.normal(key, shape, _dt.canonicalize(dtype_ or dtype) or torch.float32,
                              sharding=sharding) * stddev
    return init


def constant(value, dtype=None):
    def init(key, shape, dtype_=None, sharding=None):
        from ..array import device_put
        dt = _dt.canonicalize(dtype_ or dtype) or torch.float32
        from ..spmd.state import abstract_mode
        if abstract_mode():
            from ..sharding.shardings import default_sharding
            from ..array import ShardedArray
            sh = sharding or default_sharding()
            ta = sh.tile_assignment(len(shape))
            return ShardedArray(shape, dt, sh, {d: torch.empty(ta.shard_shape(shape), dtype=dt, device="meta")
                                                for d in ta.device_ids if _is_local(d)})
        return device_put(torch.full(tuple(shape), float(value), dtype=dt), sharding)
    return init


def _is_local(d):
    from ..runtime.devices import get_device, process_index
    return get_device(d).process_index == process_index()


def zeros(key, shape, dtype=None, sharding=None):
    return constant(0.0)(key, shape, dtype, sharding)


def ones(key, shape, dtype=None, sharding=None):
    return constant(1.0)(key, shape, dtype, sharding)


zeros_init = lambda: zeros  # noqa: E731
