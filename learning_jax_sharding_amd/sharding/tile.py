"""TileAssignment: the one sharding representation the partitioner reasons about.

Why this exists: ``case1a.py:30`` places B with
``sharding.reshape(4,2).replicate(axis=1)`` on a (2,4) device grid, which puts
contraction block ``d//2`` on device ``d`` while A holds block ``d%4``.  That
layout is not expressible as ``NamedSharding(mesh, P)`` over the (2,4) mesh, so
the core representation is GSPMD-style: an integer array of device ids with
shape ``tile_shape + (num_replicas,)``.  Element ``[t0,..,tr-1, r]`` is the
r-th device holding tile ``(t0,..,tr-1)``.  Named and positional shardings are
front-ends that lower to this.
"""
from __future__ import annotations

from functools import cached_property
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

__all__ = ["TileAssignment", "Region", "region_intersect", "region_size"]

Region = Tuple[Tuple[int, int], ...]  # per-dim [start, stop)


def region_intersect(a: Region, b: Region) -> Optional[Region]:
    out = []
    for (a0, a1), (b0, b1) in zip(a, b):
        lo, hi = max(a0, b0), min(a1, b1)
        if hi <= lo:
            return None
        out.append((lo, hi))
    return tuple(out)


def region_size(r: Optional[Region]) -> int:
    if r is None:
        return 0
    n = 1
    for lo, hi in r:
        n *= hi - lo
    return n


def region_contains(outer: Region, inner: Region) -> bool:
    return all(o0 <= i0 and i1 <= o1 for (o0, o1), (i0, i1) in zip(outer, inner))


class TileAssignment:
    """Device ids arranged as ``tile_shape + (num_replicas,)`` (canonical: replicas sorted)."""

    __slots__ = ("ids", "__dict__")

    def __init__(self, ids):
        ids = np.asarray(ids, dtype=np.int64)
        if ids.ndim < 1:
            raise ValueError("TileAssignment needs at least the replica dimension")
        self.ids = np.sort(ids, axis=-1)
        flat = self.ids.reshape(-1)
        if len(np.unique(flat)) != flat.size:
            raise ValueError(f"device appears twice in tile assignment {self.ids.tolist()}")

    # ---------------------------------------------------------------- constructors
    @staticmethod
    def replicated(device_ids: Sequence[int], ndim: int) -> "TileAssignment":
        return TileAssignment(np.asarray(sorted(device_ids), dtype=np.int64).reshape((1,) * ndim + (-1,)))

    @staticmethod
    def from_coords(coords: Dict[int, Tuple[int, ...]], tile_shape: Sequence[int]) -> Optional["TileAssignment"]:
        """Build from ``device -> tile coordinate``; None if tiles are unequally covered."""
        tile_shape = tuple(int(t) for t in tile_shape)
        n_tiles = int(np.prod(tile_shape)) if tile_shape else 1
        if len(coords) % n_tiles:
            return None
        r = len(coords) // n_tiles
        buckets: Dict[Tuple[int, ...], List[int]] = {}
        for d, c in coords.items():
            buckets.setdefault(tuple(c), []).append(d)
        if len(buckets) != n_tiles or any(len(v) != r for v in buckets.values()):
            return None
        ids = np.empty(tile_shape + (r,), dtype=np.int64)
        for c, devs in buckets.items():
            ids[c] = sorted(devs)
        return TileAssignment(ids)

    # ---------------------------------------------------------------- basic props
    @property
    def ndim(self) -> int:
        return self.ids.ndim - 1

    @property
    def tile_shape(self) -> Tuple[int, ...]:
        return tuple(self.ids.shape[:-1])

    @property
    def num_replicas(self) -> int:
        return int(self.ids.shape[-1])

    @property
    def num_devices(self) -> int:
        return int(self.ids.size)

    @cached_property
    def device_ids(self) -> Tuple[int, ...]:
        return tuple(sorted(int(x) for x in self.ids.reshape(-1)))

    @cached_property
    def coords(self) -> Dict[int, Tuple[int, ...]]:
        out = {}
        for idx in np.ndindex(*self.ids.shape):
            out[int(self.ids[idx])] = tuple(int(i) for i in idx[:-1])
        return out

    @cached_property
    def replica_index(self) -> Dict[int, int]:
        out = {}
        for idx in np.ndindex(*self.ids.shape):
            out[int(self.ids[idx])] = int(idx[-1])
        return out

    @property
    def is_fully_replicated(self) -> bool:
        return all(t == 1 for t in self.tile_shape)

    def holders(self, tile: Tuple[int, ...]) -> Tuple[int, ...]:
        return tuple(int(x) for x in self.ids[tuple(tile)])

    def sharded_dims(self) -> Tuple[int, ...]:
        return tuple(i for i, t in enumerate(self.tile_shape) if t > 1)

    # ---------------------------------------------------------------- geometry
    def check_shape(self, shape: Sequence[int]) -> None:
        if len(shape) != self.ndim:
            raise ValueError(f"sharding of rank {self.ndim} used with array of shape {tuple(shape)}")
        for s, t in zip(shape, self.tile_shape):
            if s % t:
                raise ValueError(
                    f"array shape {tuple(shape)} is not divisible by tile grid {self.tile_shape}; "
                    "uneven sharding is not supported")

    def shard_shape(self, shape: Sequence[int]) -> Tuple[int, ...]:
        self.check_shape(shape)
        return tuple(int(s) // int(t) for s, t in zip(shape, self.tile_shape))

    def tile_region(self, tile: Tuple[int, ...], shape: Sequence[int]) -> Region:
        ss = self.shard_shape(shape)
        return tuple((c * s, (c + 1) * s) for c, s in zip(tile, ss))

    def region(self, dev: int, shape: Sequence[int]) -> Region:
        return self.tile_region(self.coords[int(dev)], shape)

    def indices(self, dev: int, shape: Sequence[int]) -> Tuple[slice, ...]:
        return tuple(slice(lo, hi) for lo, hi in self.region(dev, shape))

    # ---------------------------------------------------------------- algebra
    def canonical_key(self):
        return (self.ids.shape, self.ids.tobytes())

    def __eq__(self, other):
        return isinstance(other, TileAssignment) and self.canonical_key() == other.canonical_key()

    def __hash__(self):
        return hash(self.canonical_key())

    def __repr__(self):
        return f"TileAssignment(tiles={self.tile_shape}, replicas={self.num_replicas}, ids={self.ids.tolist()})"

    def transpose(self, perm: Sequence[int]) -> "TileAssignment":
        perm = tuple(perm) + (self.ndim,)
        return TileAssignment(np.transpose(self.ids, perm))

    def project(self, dims: Sequence[int]) -> "TileAssignment":
        """Keep only ``dims`` (in that order); other dims' tiles become replicas."""
        dims = tuple(dims)
        rest = tuple(i for i in range(self.ndim) if i not in dims)
        moved = np.transpose(self.ids, dims + rest + (self.ndim,))
        kept_shape = tuple(self.ids.shape[i] for i in dims)
        return TileAssignment(moved.reshape(kept_shape + (-1,)))

    def insert_dims(self, positions: Sequence[int], new_ndim: int) -> "TileAssignment":
        """Insert unsharded (tile count 1) dims so the result has rank ``new_ndim``.

        ``positions`` are the output positions of the existing dims, in order.
        """
        shape = [1] * new_ndim
        for src, dst in enumerate(positions):
            shape[dst] = self.tile_shape[src]
        # existing dims keep their order, so a reshape suffices
        return TileAssignment(self.ids.reshape(tuple(shape) + (self.num_replicas,)))

    def unshard(self, dims: Iterable[int]) -> "TileAssignment":
        """Same grouping, but ``dims`` become unsharded (their tiles merge into replicas)."""
        dims = set(dims)
        keep = tuple(i for i in range(self.ndim) if i not in dims)
        proj = self.project(keep)
        return proj.insert_dims(keep, self.ndim)

    def with_device_order(self) -> List[int]:
        return list(self.device_ids)

    def groups_along(self, dims: Sequence[int]) -> List[Tuple[int, ...]]:
        """Partition devices into groups that each hold every tile of ``dims`` exactly once.

        Members of a group share all other tile coordinates and the same replica
        slot; members are ordered by their (row-major) tile index over ``dims``.
        This is the device group of an all-gather / all-reduce / all-to-all over
        ``dims``.
        """
        dims = tuple(dims)
        rest = tuple(i for i in range(self.ndim) if i not in dims)
        moved = np.transpose(self.ids, rest + dims + (self.ndim,))
        n_rest = int(np.prod([self.ids.shape[i] for i in rest])) if rest else 1
        n_g = int(np.prod([self.ids.shape[i] for i in dims])) if dims else 1
        moved = moved.reshape(n_rest, n_g, self.num_replicas)
        groups = []
        for a in range(n_rest):
            for r in range(self.num_replicas):
                groups.append(tuple(int(x) for x in moved[a, :, r]))
        return groups
