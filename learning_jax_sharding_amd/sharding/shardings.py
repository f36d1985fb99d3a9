"""Sharding front-ends: PartitionSpec, NamedSharding, PositionalSharding, GSPMD, single-device.

Reference surface:
* ``PositionalSharding(mesh_utils.create_device_mesh((2,4)))`` - ``case1a.py:15``;
  ``.replicate(axis, keepdims=True)`` - ``case1a.py:24``; ``.reshape(4,2)`` -
  ``case1a.py:30``.
* ``NamedSharding(mesh, PartitionSpec('data','model'))`` - ``case6_attention.py:158-161``;
  ``PartitionSpec(None)`` / ``mesh_sharding(None)`` - ``case6_attention.py:193``.

Every class lowers to :class:`TileAssignment` for a given array rank.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..mesh import Mesh
from ..runtime.devices import Device, get_device, process_index
from .tile import TileAssignment

__all__ = [
    "PartitionSpec",
    "P",
    "Sharding",
    "NamedSharding",
    "PositionalSharding",
    "GSPMDSharding",
    "SingleDeviceSharding",
    "sharding_from_tile",
]


class PartitionSpec(tuple):
    """Per-dimension mesh axes: ``None`` (replicated), an axis name, or a tuple of names.

    Shorter than the array rank means trailing dims are replicated.
    """

    __pytree_leaf__ = True  # a spec is a leaf of sharding trees, not a container

    def __new__(cls, *parts):
        norm = []
        for p in parts:
            if isinstance(p, list):
                p = tuple(p)
            if isinstance(p, tuple) and len(p) == 1:
                p = p[0]
            if isinstance(p, tuple) and len(p) == 0:
                p = None
            norm.append(p)
        return tuple.__new__(cls, norm)

    def __repr__(self):
        return "PartitionSpec(" + ", ".join(repr(p) for p in self) + ")"

    def axes_for_dim(self, i: int) -> Tuple[str, ...]:
        if i >= len(self):
            return ()
        p = self[i]
        if p is None:
            return ()
        if isinstance(p, str):
            return (p,)
        return tuple(p)

    def __reduce__(self):
        return (PartitionSpec, tuple(self))


P = PartitionSpec


class Sharding:
    """Base class.  Subclasses implement :meth:`tile_assignment` and ``_device_assignment``."""

    def tile_assignment(self, ndim: int) -> TileAssignment:
        raise NotImplementedError

    @property
    def _device_assignment(self) -> Tuple[Device, ...]:
        raise NotImplementedError

    @property
    def device_set(self):
        return set(self._device_assignment)

    @property
    def addressable_devices(self):
        pi = process_index()
        return {d for d in self._device_assignment if d.process_index == pi}

    @property
    def is_fully_addressable(self) -> bool:
        pi = process_index()
        return all(d.process_index == pi for d in self._device_assignment)

    def is_fully_replicated_for(self, ndim: int) -> bool:
        return self.tile_assignment(ndim).is_fully_replicated

    @property
    def is_fully_replicated(self) -> bool:  # rank independent for all front-ends used here
        return self.tile_assignment(self._natural_ndim()).is_fully_replicated

    def _natural_ndim(self) -> int:
        return 0

    def shard_shape(self, global_shape: Sequence[int]) -> Tuple[int, ...]:
        return self.tile_assignment(len(global_shape)).shard_shape(global_shape)

    def devices_indices_map(self, global_shape: Sequence[int]) -> Dict[Device, Tuple[slice, ...]]:
        ta = self.tile_assignment(len(global_shape))
        return {get_device(d): ta.indices(d, global_shape) for d in ta.device_ids}

    def is_equivalent_to(self, other: "Sharding", ndim: int) -> bool:
        return self.tile_assignment(ndim) == other.tile_assignment(ndim)


class NamedSharding(Sharding):
    def __init__(self, mesh: Mesh, spec: PartitionSpec = PartitionSpec()):
        if spec is None:
            spec = PartitionSpec()
        if not isinstance(spec, PartitionSpec):
            spec = PartitionSpec(*spec) if isinstance(spec, (tuple, list)) else PartitionSpec(spec)
        used = []
        for i in range(len(spec)):
            for a in spec.axes_for_dim(i):
                if a not in mesh.axis_names:
                    raise ValueError(f"PartitionSpec {spec} names axis {a!r} not in mesh {mesh.axis_names}")
                if a in used:
                    raise ValueError(f"mesh axis {a!r} used twice in {spec}")
                used.append(a)
        self.mesh = mesh
        self.spec = spec
        self._cache: Dict[int, TileAssignment] = {}

    def tile_assignment(self, ndim: int) -> TileAssignment:
        ta = self._cache.get(ndim)
        if ta is not None:
            return ta
        if len(self.spec) > ndim:
            raise ValueError(f"{self.spec} has more entries than array rank {ndim}")
        ids = self.mesh.device_ids
        names = list(self.mesh.axis_names)
        order: List[int] = []
        tiles: List[int] = []
        for i in range(ndim):
            axes = self.spec.axes_for_dim(i)
            n = 1
            for a in axes:
                k = names.index(a)
                order.append(k)
                n *= ids.shape[k]
            tiles.append(n)
        rest = [k for k in range(len(names)) if k not in order]
        moved = np.transpose(ids, order + rest) if names else ids
        ta = TileAssignment(np.asarray(moved).reshape(tuple(tiles) + (-1,)))
        self._cache[ndim] = ta
        return ta

    @property
    def _device_assignment(self):
        return tuple(self.mesh.devices.flat)

    def _natural_ndim(self):
        return len(self.spec)

    def __repr__(self):
        return f"NamedSharding(mesh={dict(self.mesh.shape)}, spec={self.spec})"

    def __eq__(self, other):
        return isinstance(other, NamedSharding) and other.mesh == self.mesh and tuple(other.spec) == tuple(self.spec)

    def __hash__(self):
        return hash((self.mesh, tuple(self.spec)))


class PositionalSharding(Sharding):
    """A device grid whose rank equals the array rank; cells may hold device *sets*.

    Internally ``_ids`` has shape ``grid_shape + (set_size,)``.
    """

    def __init__(self, devices, *, _ids=None, _devices=None):
        if _ids is not None:
            self._ids = np.asarray(_ids, dtype=np.int64)
            self._devices = tuple(_devices)
            return
        arr = np.asarray(devices, dtype=object)
        if isinstance(devices, Device):
            arr = np.asarray([devices], dtype=object).reshape(())
        self._devices = tuple(arr.flat)
        ids = np.vectorize(lambda d: d.id, otypes=[np.int64])(arr) if arr.size else np.zeros(arr.shape, np.int64)
        self._ids = ids[..., None]

    @property
    def shape(self) -> Tuple[int, ...]:
        return tuple(self._ids.shape[:-1])

    @property
    def ndim(self) -> int:
        return self._ids.ndim - 1

    def _with(self, ids) -> "PositionalSharding":
        return PositionalSharding(None, _ids=ids, _devices=self._devices)

    def reshape(self, *shape) -> "PositionalSharding":
        if len(shape) == 1 and isinstance(shape[0], (tuple, list)):
            shape = tuple(shape[0])
        return self._with(self._ids.reshape(tuple(shape) + (self._ids.shape[-1],)))

    def transpose(self, *axes) -> "PositionalSharding":
        if not axes:
            axes = tuple(reversed(range(self.ndim)))
        elif len(axes) == 1 and isinstance(axes[0], (tuple, list)):
            axes = tuple(axes[0])
        return self._with(np.transpose(self._ids, tuple(axes) + (self.ndim,)))

    @property
    def T(self):
        return self.transpose()

    def replicate(self, axis=None, keepdims: bool = True) -> "PositionalSharding":
        """Merge grid axis ``axis`` into the device sets (``case1a.py:24``)."""
        ids = self._ids
        if axis is None:
            axes = tuple(range(self.ndim))
        else:
            axes = (axis,) if isinstance(axis, int) else tuple(axis)
            axes = tuple(a % self.ndim for a in axes)
        keep = tuple(i for i in range(self.ndim) if i not in axes)
        moved = np.transpose(ids, keep + axes + (self.ndim,))
        kshape = tuple(ids.shape[i] for i in keep)
        merged = np.sort(moved.reshape(kshape + (-1,)), axis=-1)
        if keepdims:
            full = [1] * self.ndim
            for i in keep:
                full[i] = ids.shape[i]
            merged = merged.reshape(tuple(full) + (merged.shape[-1],))
        return self._with(merged)

    def tile_assignment(self, ndim: int) -> TileAssignment:
        if self.ndim != ndim:
            raise ValueError(
                f"PositionalSharding of rank {self.ndim} (shape {self.shape}) cannot shard a rank-{ndim} array")
        return TileAssignment(self._ids)

    @property
    def _device_assignment(self):
        return self._devices

    def _natural_ndim(self):
        return self.ndim

    def __repr__(self):
        return f"PositionalSharding({self._ids.tolist()})"

    def __eq__(self, other):
        return isinstance(other, PositionalSharding) and np.array_equal(other._ids, self._ids)

    def __hash__(self):
        return hash((self._ids.shape, self._ids.tobytes()))


class GSPMDSharding(Sharding):
    """A raw tile assignment (op outputs that match no friendlier front-end)."""

    def __init__(self, devices: Sequence[Device], tile: TileAssignment):
        self._devices = tuple(devices)
        self.tile = tile

    def tile_assignment(self, ndim: int) -> TileAssignment:
        if ndim != self.tile.ndim:
            raise ValueError(f"GSPMDSharding of rank {self.tile.ndim} used for rank {ndim}")
        return self.tile

    @property
    def _device_assignment(self):
        return self._devices

    def _natural_ndim(self):
        return self.tile.ndim

    def __repr__(self):
        return f"GSPMDSharding({self.tile!r})"

    def __eq__(self, other):
        return isinstance(other, GSPMDSharding) and other.tile == self.tile

    def __hash__(self):
        return hash(self.tile)


class SingleDeviceSharding(Sharding):
    def __init__(self, device: Device):
        self.device = device

    def tile_assignment(self, ndim: int) -> TileAssignment:
        return TileAssignment.replicated([self.device.id], ndim)

    @property
    def _device_assignment(self):
        return (self.device,)

    def __repr__(self):
        return f"SingleDeviceSharding(device={self.device!r})"

    def __eq__(self, other):
        return isinstance(other, SingleDeviceSharding) and other.device == self.device

    def __hash__(self):
        return hash(("single", self.device.id))


class ReplicatedSharding(Sharding):
    """Every device holds the whole array (rank independent)."""

    def __init__(self, devices: Sequence[Device]):
        self._devices = tuple(devices)

    def tile_assignment(self, ndim: int) -> TileAssignment:
        return TileAssignment.replicated([d.id for d in self._devices], ndim)

    @property
    def _device_assignment(self):
        return self._devices

    def __repr__(self):
        return f"ReplicatedSharding({[d.id for d in self._devices]})"

    def __eq__(self, other):
        return isinstance(other, ReplicatedSharding) and other._devices == self._devices

    def __hash__(self):
        return hash(("repl", tuple(d.id for d in self._devices)))


def default_sharding() -> Sharding:
    """Where unplaced arrays live: device 0 (JAX's default device) in one process; replicated
    on every device when one process drives each GPU (each rank computes its own copy)."""
    from ..runtime.devices import devices, is_distributed
    from ..spmd.state import default_placement
    placed = default_placement()
    if placed is not None:
        return placed
    devs = devices()
    if is_distributed():
        return ReplicatedSharding(devs)
    return SingleDeviceSharding(devs[0])


def sharding_from_tile(tile: TileAssignment, like: Sequence[Sharding] = ()) -> Sharding:
    """Pick the friendliest front-end for ``tile``.

    If one of ``like`` is a NamedSharding whose mesh can express ``tile`` with a
    PartitionSpec, return that NamedSharding; a single device becomes a
    SingleDeviceSharding; otherwise a GSPMDSharding whose device order follows
    the first of ``like`` (this keeps ``device_buffers`` in mesh order).
    """
    devs_in_tile = set(tile.device_ids)
    for s in like:
        if isinstance(s, NamedSharding) and set(d.id for d in s.mesh.devices.flat) == devs_in_tile:
            spec = _find_spec(s.mesh, tile)
            if spec is not None:
                return NamedSharding(s.mesh, spec)
    if len(devs_in_tile) == 1:
        return SingleDeviceSharding(get_device(next(iter(devs_in_tile))))
    order: Tuple[Device, ...] = ()
    for s in like:
        if set(d.id for d in s._device_assignment) == devs_in_tile:
            order = tuple(s._device_assignment)
            break
    if not order:
        order = tuple(get_device(d) for d in sorted(devs_in_tile))
    return GSPMDSharding(order, tile)


def _find_spec(mesh: Mesh, tile: TileAssignment) -> Optional[PartitionSpec]:
    """Search assignments of mesh axes to array dims reproducing ``tile`` (small meshes only)."""
    import itertools

    names = mesh.axis_names
    sizes = dict(mesh.shape)
    nd = tile.ndim
    # candidate axis tuples per dim whose product equals the tile count
    per_dim: List[List[Tuple[str, ...]]] = []
    for i, t in enumerate(tile.tile_shape):
        cands = []
        for r in range(0, len(names) + 1):
            for combo in itertools.permutations(names, r):
                if int(np.prod([sizes[a] for a in combo])) == t:
                    cands.append(combo)
        if not cands:
            return None
        per_dim.append(cands)
    for choice in itertools.product(*per_dim):
        flat = [a for c in choice for a in c]
        if len(flat) != len(set(flat)):
            continue
        spec = PartitionSpec(*[(c if len(c) > 1 else (c[0] if c else None)) for c in choice])
        # trim trailing Nones for readability
        parts = list(spec)
        while parts and parts[-1] is None:
            parts.pop()
        spec = PartitionSpec(*parts)
        try:
            if NamedSharding(mesh, spec).tile_assignment(nd) == tile:
                return spec
        except ValueError:
            continue
    return None
