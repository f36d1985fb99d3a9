"""Global-view sharded arrays.

A :class:`ShardedArray` is a global shape + dtype + :class:`Sharding` plus the
torch tensors of its *addressable* shards (all of them in single-process mode;
the local GPU's shard in the one-process-per-GPU RCCL mode).

Reference surface: ``jax.device_put(x, sharding)`` (``case1a.py:24``),
``.device_buffers[i]`` (``case1a.py:35``), ``.addressable_shards[i].data``
(``case4_gspmd_ff.py:56``), ``np.array(arr)`` (``case1a.py:62``).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import dtypes as _dt
from .runtime.devices import Device, devices as _all_devices, get_device, process_index
from .sharding.shardings import Sharding, SingleDeviceSharding
from .sharding.tile import TileAssignment

__all__ = ["ShardedArray", "Shard", "device_put", "is_array", "ShapeDtypeStruct"]


class ShapeDtypeStruct:
    """Abstract array (what ``eval_shape`` returns)."""

    def __init__(self, shape, dtype, sharding: Optional[Sharding] = None):
        self.shape = tuple(int(s) for s in shape)
        self.dtype = _dt.canonicalize(dtype)
        self.sharding = sharding

    @property
    def ndim(self):
        return len(self.shape)

    @property
    def size(self):
        return int(np.prod(self.shape)) if self.shape else 1

    def __repr__(self):
        return f"ShapeDtypeStruct(shape={self.shape}, dtype={str(self.dtype).replace('torch.', '')})"

    def __eq__(self, other):
        return isinstance(other, ShapeDtypeStruct) and other.shape == self.shape and other.dtype == self.dtype

    def __hash__(self):
        return hash((self.shape, self.dtype))


class Shard:
    def __init__(self, device: Device, index: Tuple[slice, ...], replica_id: int, data: "ShardedArray"):
        self.device = device
        self.index = index
        self.replica_id = replica_id
        self.data = data

    def __repr__(self):
        return f"Shard(device={self.device!r}, index={self.index}, replica_id={self.replica_id})"


class LazyLocal(dict):
    """Per-device tensors computed on first use: ``thunk()`` returns the {device: tensor} dict.

    Used for values a training step usually never reads -- the all-reduced scalar loss of
    ``grad`` (its gradient is seeded on the pre-reduction partial sums): the collective that
    would produce it runs only if something reads the value, the way XLA drops the primal
    output of ``jax.grad``.  Every dict access materialises it."""

    def __init__(self, thunk):
        super().__init__()
        self._thunk = thunk

    def _force(self):
        if self._thunk is not None:
            th, self._thunk = self._thunk, None
            super().update(th())
        return self

    @property
    def pending(self) -> bool:
        return self._thunk is not None

    def __getitem__(self, k):
        return dict.__getitem__(self._force(), k)

    def __iter__(self):
        return dict.__iter__(self._force())

    def __len__(self):
        return dict.__len__(self._force())

    def __contains__(self, k):
        return dict.__contains__(self._force(), k)

    def keys(self):
        return dict.keys(self._force())

    def values(self):
        return dict.values(self._force())

    def items(self):
        return dict.items(self._force())

    def get(self, k, default=None):
        return dict.get(self._force(), k, default)

    def copy(self):
        return dict(self._force())

    def __repr__(self):
        return "LazyLocal(<pending>)" if self._thunk is not None else dict.__repr__(self)


class ShardedArray:
    __array_priority__ = 100

    def __init__(self, shape: Sequence[int], dtype, sharding: Sharding, local: Dict[int, torch.Tensor]):
        self.shape = tuple(int(s) for s in shape)
        self.dtype = _dt.canonicalize(dtype)
        self.sharding = sharding
        self.local = local if isinstance(local, LazyLocal) and local.pending else dict(local)
        self._tile: Optional[TileAssignment] = None

    # ------------------------------------------------------------------ metadata
    @property
    def tile(self) -> TileAssignment:
        if self._tile is None:
            self._tile = self.sharding.tile_assignment(len(self.shape))
        return self._tile

    @property
    def ndim(self) -> int:
        return len(self.shape)

    @property
    def size(self) -> int:
        return int(np.prod(self.shape)) if self.shape else 1

    @property
    def nbytes(self) -> int:
        return self.size * _dt.itemsize(self.dtype)

    def __len__(self):
        if not self.shape:
            raise TypeError("len() of unsized object")
        return self.shape[0]

    @property
    def is_fully_replicated(self) -> bool:
        return self.tile.is_fully_replicated

    @property
    def is_fully_addressable(self) -> bool:
        return self.sharding.is_fully_addressable

    @property
    def weak_type(self):
        return False

    def local_tensors(self) -> List[torch.Tensor]:
        return [self.local[d] for d in sorted(self.local)]

    # ------------------------------------------------------------------ shards
    def _ordered_addressable(self) -> List[Device]:
        pi = process_index()
        return [d for d in self.sharding._device_assignment if d.process_index == pi and d.id in self.local]

    @property
    def device_buffers(self) -> List["ShardedArray"]:
        out = []
        for d in self._ordered_addressable():
            t = self.local[d.id]
            out.append(ShardedArray(t.shape, self.dtype, SingleDeviceSharding(d), {d.id: t}))
        return out

    @property
    def addressable_shards(self) -> List[Shard]:
        out = []
        ta = self.tile
        for d in self._ordered_addressable():
            t = self.local[d.id]
            data = ShardedArray(t.shape, self.dtype, SingleDeviceSharding(d), {d.id: t})
            out.append(Shard(d, ta.indices(d.id, self.shape), ta.replica_index[d.id], data))
        return out

    def addressable_data(self, i: int) -> "ShardedArray":
        return self.addressable_shards[i].data

    def devices(self):
        return self.sharding.device_set

    # ------------------------------------------------------------------ host transfer
    def to_torch(self, device: Optional[torch.device] = None) -> torch.Tensor:
        """Assemble the global value as one torch tensor (host by default)."""
        if not self.is_fully_addressable:
            from .utils.multihost import process_allgather
            return process_allgather(self, device=device)
        device = torch.device("cpu") if device is None else device
        ta = self.tile
        if len(self.local) == 1 or ta.is_fully_replicated:
            d = next(iter(self.local)) if ta.is_fully_replicated else None
            if d is not None:
                return self.local[d].detach().to(device)
        out = torch.empty(self.shape, dtype=self.dtype, device=device)
        done = set()
        for d in sorted(self.local):
            tile = ta.coords[d]
            if tile in done:
                continue
            done.add(tile)
            out[ta.indices(d, self.shape)] = self.local[d].detach().to(device)
        return out

    def __array__(self, dtype=None, copy=None):
        t = self.to_torch()
        if t.dtype in (torch.bfloat16, torch.float8_e4m3fn, torch.float8_e5m2):
            t = t.float()
        a = t.numpy()
        if dtype is not None:
            a = a.astype(dtype)
        return a

    def tolist(self):
        return np.asarray(self).tolist()

    def item(self):
        return np.asarray(self).item()

    def __float__(self):
        return float(self.item())

    def __int__(self):
        return int(self.item())

    def __bool__(self):
        return bool(self.item())

    def block_until_ready(self) -> "ShardedArray":
        for t in self.local.values():
            if t.is_cuda:
                torch.cuda.synchronize(t.device)
                break
        return self

    def __repr__(self):
        dt = str(self.dtype).replace("torch.", "")
        if self.is_fully_addressable and self.size <= 64 and not any(t.is_meta for t in self.local.values()):
            return f"Array({np.asarray(self)!r}, dtype={dt})".replace("array(", "").replace("\n      ", "\n")
        return f"Array(shape={self.shape}, dtype={dt}, sharding={self.sharding!r})"

    # ------------------------------------------------------------------ ops (global view)
    def astype(self, dtype) -> "ShardedArray":
        from .ops import core
        return core.convert(self, dtype)

    def reshape(self, *shape) -> "ShardedArray":
        from .ops import core
        if len(shape) == 1 and isinstance(shape[0], (tuple, list)):
            shape = tuple(shape[0])
        return core.reshape(self, shape)

    def transpose(self, *axes) -> "ShardedArray":
        from .ops import core
        if not axes:
            axes = tuple(reversed(range(self.ndim)))
        elif len(axes) == 1 and isinstance(axes[0], (tuple, list)):
            axes = tuple(axes[0])
        return core.transpose(self, axes)

    @property
    def T(self):
        return self.transpose()

    def sum(self, axis=None, keepdims=False, dtype=None):
        from .ops import core
        return core.reduce_sum(self, axis, keepdims=keepdims, dtype=dtype)

    def mean(self, axis=None, keepdims=False):
        from .ops import core
        return core.reduce_mean(self, axis, keepdims=keepdims)

    def max(self, axis=None, keepdims=False):
        from .ops import core
        return core.reduce_max(self, axis, keepdims=keepdims)

    def __getitem__(self, idx):
        from .ops import core
        return core.getitem(self, idx)

    def _bin(self, other, op, reverse=False):
        from .ops import core
        return core.binary(op, other, self) if reverse else core.binary(op, self, other)

    def __add__(self, o):
        return self._bin(o, "add")

    def __radd__(self, o):
        return self._bin(o, "add", True)

    def __sub__(self, o):
        return self._bin(o, "sub")

    def __rsub__(self, o):
        return self._bin(o, "sub", True)

    def __mul__(self, o):
        return self._bin(o, "mul")

    def __rmul__(self, o):
        return self._bin(o, "mul", True)

    def __truediv__(self, o):
        return self._bin(o, "div")

    def __rtruediv__(self, o):
        return self._bin(o, "div", True)

    def __pow__(self, o):
        return self._bin(o, "pow")

    def __neg__(self):
        from .ops import core
        return core.unary("neg", self)

    def __matmul__(self, o):
        from .ops import core
        return core.matmul(self, o)

    def __rmatmul__(self, o):
        from .ops import core
        return core.matmul(o, self)


def is_array(x) -> bool:
    return isinstance(x, ShardedArray)


def _as_host_tensor(x) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x
    if isinstance(x, np.ndarray):
        if x.dtype == np.float64:
            x = x.astype(np.float32)  # JAX default (x64 disabled)
        if x.dtype == np.int64:
            x = x.astype(np.int32)
        return torch.from_numpy(np.ascontiguousarray(x))
    if isinstance(x, (float, int, bool)):
        return torch.tensor(x, dtype=_dt.canonicalize(type(x)))
    return _as_host_tensor(np.asarray(x))


def _place_global(t: torch.Tensor, sharding: Sharding, dtype=None) -> ShardedArray:
    dtype = _dt.canonicalize(dtype) or t.dtype
    shape = tuple(t.shape)
    ta = sharding.tile_assignment(len(shape))
    ta.check_shape(shape)
    pi = process_index()
    local = {}
    for d in ta.device_ids:
        dev = get_device(d)
        if dev.process_index != pi:
            continue
        piece = t[ta.indices(d, shape)]
        local[d] = piece.to(device=dev.torch_device, dtype=dtype, copy=True).contiguous()
    return ShardedArray(shape, dtype, sharding, local)


def device_put(x, device=None, *, may_alias=None, donate=None):
    """Place ``x`` (host value, torch tensor or ShardedArray, or a pytree of them).

    ``device`` may be a :class:`Device`, a :class:`Sharding` or None (device 0).
    A ShardedArray input is resharded with collectives (no host round trip).
    """
    from .utils import tree as _tree

    if not isinstance(x, ShardedArray) and _tree.is_container(x):
        if isinstance(device, (list, tuple)) or _tree.is_container(device):
            return _tree.tree_map(lambda a, s: device_put(a, s), x, device)
        return _tree.tree_map(lambda a: device_put(a, device), x)
    if device is None:
        from .sharding.shardings import default_sharding
        sharding = default_sharding()
    elif isinstance(device, Device):
        sharding = SingleDeviceSharding(device)
    elif isinstance(device, Sharding):
        sharding = device
    else:
        raise TypeError(f"device_put target must be a Device or Sharding, got {type(device)}")
    if isinstance(x, ShardedArray):
        from .spmd.reshard import reshard
        return reshard(x, sharding)
    return _place_global(_as_host_tensor(x), sharding)
