"""Counter-based random numbers (``jax.random`` subset), shard-invariant.

Reference usage: ``jax.random.PRNGKey(0)`` / ``jax.random.key(0)`` and
``jax.random.normal(key, shape)`` (``case1a.py:16-18``, ``case6_attention.py:147,152``);
``nn.initializers.lecun_normal()`` (truncated normal) for parameters
(``case6_attention.py:57``).

Design: Philox4x32-10.  Element ``i`` of an array (row-major global index) is
a pure function of ``(key, i)``, so every device generates exactly its own
shard (no full-array materialisation, no communication) and values do not
depend on the mesh.  Bit-exact parity with JAX's threefry is not a goal
(SURVEY §2.2); the reference's quirk that A and B drawn with the same key and
the same element count are equal (``case1a.py:17-18``) does hold.

The GPU path is the ``ljs_rng_*`` HIP kernels; host devices use the numpy
implementation below (same integer stream; floats agree to a few ulps).
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import numpy as np
import torch

from . import dtypes as _dt
from .array import ShardedArray
from .runtime.devices import devices as _devices, get_device, process_index
from .sharding.shardings import Sharding, SingleDeviceSharding

__all__ = ["PRNGKey", "key", "split", "fold_in", "normal", "uniform", "truncated_normal", "bits", "Key",
           "key_data"]

_M0, _M1 = 0xD2511F53, 0xCD9E8D57
_W0, _W1 = 0x9E3779B9, 0xBB67AE85
_MASK = 0xFFFFFFFF


class Key:
    """A PRNG key: two uint32 words (host-side; keys never need to live on a device)."""

    __slots__ = ("k0", "k1")

    def __init__(self, k0: int, k1: int):
        self.k0 = int(k0) & _MASK
        self.k1 = int(k1) & _MASK

    @property
    def shape(self):
        return ()

    def __repr__(self):
        return f"Key([{self.k0}, {self.k1}])"

    def __eq__(self, other):
        return isinstance(other, Key) and (self.k0, self.k1) == (other.k0, other.k1)

    def __hash__(self):
        return hash((self.k0, self.k1))

    def __iter__(self):
        yield self.k0
        yield self.k1


def PRNGKey(seed: int) -> Key:
    seed = int(seed)
    return Key(seed & _MASK, (seed >> 32) & _MASK)


def key(seed: int) -> Key:
    return PRNGKey(seed)


def key_data(k: Key) -> np.ndarray:
    return np.array([k.k0, k.k1], dtype=np.uint32)


# ----------------------------------------------------------------------------- philox (numpy)
def _philox_np(ctr_lo: np.ndarray, ctr_hi: np.ndarray, k0: int, k1: int, c2: int = 0, c3: int = 0):
    c0 = ctr_lo.astype(np.uint64)
    c1 = ctr_hi.astype(np.uint64)
    c2 = np.full_like(c0, c2)
    c3 = np.full_like(c0, c3)
    key0 = np.uint64(k0)
    key1 = np.uint64(k1)
    m0, m1, mask = np.uint64(_M0), np.uint64(_M1), np.uint64(_MASK)
    for r in range(10):
        p0 = c0 * m0
        p1 = c2 * m1
        hi0, lo0 = p0 >> np.uint64(32), p0 & mask
        hi1, lo1 = p1 >> np.uint64(32), p1 & mask
        c0, c1, c2, c3 = (hi1 ^ c1 ^ key0) & mask, lo1, (hi0 ^ c3 ^ key1) & mask, lo0
        key0 = (key0 + np.uint64(_W0)) & mask
        key1 = (key1 + np.uint64(_W1)) & mask
    return c0, c1, c2, c3


def _philox_scalar(c0, c1, k0, k1, c2=0, c3=0):
    out = _philox_np(np.array([c0], np.uint64), np.array([c1], np.uint64), k0, k1, c2, c3)
    return tuple(int(o[0]) for o in out)


def split(k: Key, num: int = 2):
    """Derive ``num`` independent keys (philox of the key under a distinct stream id)."""
    outs = []
    for i in range(num):
        o = _philox_scalar(i, 0, k.k0, k.k1, 0x5EED, 0x51)
        outs.append(Key(o[0], o[1]))
    return outs


def fold_in(k: Key, data: int) -> Key:
    o = _philox_scalar(int(data) & _MASK, (int(data) >> 32) & _MASK, k.k0, k.k1, 0xF01D, 0x1)
    return Key(o[0], o[1])


def _u01(x: np.ndarray) -> np.ndarray:
    # 24 random bits -> (0, 1), never 0 (log-safe); exact in f32
    return ((x >> np.uint64(8)).astype(np.float64) + 0.5) * (1.0 / 16777216.0)


_SQRT2 = math.sqrt(2.0)


def _dist_np(idx: np.ndarray, k: Key, dist: str, lo: float, hi: float) -> np.ndarray:
    o0, o1, o2, o3 = _philox_np(idx & np.uint64(_MASK), idx >> np.uint64(32), k.k0, k.k1)
    if dist == "normal":
        u1, u2 = _u01(o0), _u01(o1)
        return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * math.pi * u2)
    if dist == "uniform":
        return lo + (hi - lo) * _u01(o0)
    if dist == "truncated_normal":
        from scipy.special import erf, erfinv
        a, b = erf(lo / _SQRT2), erf(hi / _SQRT2)
        u = a + (b - a) * _u01(o0)
        return np.clip(_SQRT2 * erfinv(u), lo, hi)
    if dist == "bits":
        return o0
    raise ValueError(dist)


def _generate(k: Key, shape, dtype, sharding: Optional[Sharding], dist: str, lo=0.0, hi=1.0) -> ShardedArray:
    if not isinstance(k, Key):
        raise TypeError(f"expected a PRNG key from random.PRNGKey/key, got {type(k)}")
    shape = tuple(int(s) for s in shape)
    dtype = _dt.canonicalize(dtype) if dtype is not None else torch.float32
    if sharding is None:
        from .sharding.shardings import default_sharding
        sharding = default_sharding()
    ta = sharding.tile_assignment(len(shape))
    ta.check_shape(shape)
    pi = process_index()
    local = {}
    strides = [1] * len(shape)
    for i in range(len(shape) - 2, -1, -1):
        strides[i] = strides[i + 1] * shape[i + 1]
    from .spmd.state import abstract_mode
    abstract = abstract_mode()
    for d in ta.device_ids:
        dev = get_device(d)
        if dev.process_index != pi:
            continue
        region = ta.region(d, shape)
        if abstract:
            local[d] = torch.empty(ta.shard_shape(shape), dtype=dtype if dist != "bits" else torch.int64,
                                   device="meta")
            continue
        if dev.torch_device.type == "cuda":
            from .ops import hip
            local[d] = hip.rng_fill(shape, region, k.k0, k.k1, dist, lo, hi, dtype, dev.torch_device)
            continue
        axes = [np.arange(r0, r1, dtype=np.uint64) for r0, r1 in region]
        if axes:
            grids = np.meshgrid(*axes, indexing="ij")
            idx = np.zeros(grids[0].shape, np.uint64)
            for g, s in zip(grids, strides):
                idx += g * np.uint64(s)
        else:
            idx = np.zeros((), np.uint64)
        vals = _dist_np(np.atleast_1d(idx), k, dist, lo, hi).reshape(idx.shape)
        t = torch.from_numpy(np.asarray(vals, dtype=np.float32 if dist != "bits" else np.int64))
        local[d] = t.to(dtype) if dist != "bits" else t.to(torch.int64)
    return ShardedArray(shape, dtype if dist != "bits" else torch.int64, sharding, local)


def normal(key: Key, shape: Sequence[int] = (), dtype=None, *, sharding: Optional[Sharding] = None) -> ShardedArray:
    return _generate(key, shape, dtype, sharding, "normal")


def uniform(key: Key, shape: Sequence[int] = (), dtype=None, minval: float = 0.0, maxval: float = 1.0, *,
            sharding: Optional[Sharding] = None) -> ShardedArray:
    return _generate(key, shape, dtype, sharding, "uniform", float(minval), float(maxval))


def truncated_normal(key: Key, lower: float, upper: float, shape: Sequence[int] = (), dtype=None, *,
                     sharding: Optional[Sharding] = None) -> ShardedArray:
    return _generate(key, shape, dtype, sharding, "truncated_normal", float(lower), float(upper))


def bits(key: Key, shape: Sequence[int] = (), *, sharding: Optional[Sharding] = None) -> ShardedArray:
    return _generate(key, shape, torch.int64, sharding, "bits")
