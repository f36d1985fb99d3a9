"""Reshard planner: move a ShardedArray from one tile assignment to another.

Plans are picked in order of preference; each is exact-bytes or close:

1. ``noop``        - same tile assignment.
2. ``slice``       - every device's target region lies inside what it holds
                     (replicated -> sharded): local slicing, no communication.
3. ``all_to_all``  - one dim un-shards while another dim shards over the same
                     device groups (e.g. the case6 out-projection M->S reshard,
                     ``case6_attention.py:141``).
4. ``all_gather``  - gather the dims whose target regions exceed the held
                     regions over device groups, then slice locally.
5. ``collective_permute`` - same tile grid, different placement (case1a's B,
                     ``case1a.py:30``): point-to-point tile moves.
6. ``exchange``    - general: each device pulls exactly the sub-blocks it is
                     missing from their nearest holders (point-to-point).

The all-gather plan is only chosen when it moves no more bytes than the
point-to-point exchange would (on a fully connected xGMI node a
point-to-point exchange of exactly the missing bytes is otherwise optimal).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..array import ShardedArray
from ..comm import collectives as C
from ..comm.backend import Transfer
from ..runtime.devices import get_device, process_index
from ..sharding.shardings import Sharding, sharding_from_tile
from ..sharding.tile import TileAssignment, region_contains, region_intersect, region_size
from . import plan as _plan

__all__ = ["reshard", "reshard_tile", "plan_reshard", "ReshardPlan", "reshard_cost"]


class ReshardPlan:
    def __init__(self, kind: str, **info):
        self.kind = kind
        self.info = info

    def __repr__(self):
        return f"ReshardPlan({self.kind}, {self.info})"


def _rel(region, base):
    return tuple(slice(lo - b0, hi - b0) for (lo, hi), (b0, _) in zip(region, base))


def _exchange_transfers(shape, src: TileAssignment, dst: TileAssignment) -> List[Transfer]:
    load: Dict[int, int] = {}
    transfers: List[Transfer] = []
    ss = src.shard_shape(shape)
    src_tiles = sorted(set(src.coords.values()))
    for d in dst.device_ids:
        need = dst.region(d, shape)
        for t in src_tiles:
            treg = src.tile_region(t, shape)
            inter = region_intersect(need, treg)
            if inter is None:
                continue
            holders = src.holders(t)
            if d in holders:
                h = d
            else:
                # least-loaded holder; ties broken toward the same replica slot for locality
                h = min(holders, key=lambda x: (load.get(x, 0), x))
            load[h] = load.get(h, 0) + region_size(inter)
            transfers.append(Transfer(d, h, _rel(inter, treg), _rel(inter, need)))
    return transfers


def _exchange_bytes(shape, src, dst) -> int:
    moved = 0
    for d in dst.device_ids:
        need = dst.region(d, shape)
        have = src.region(d, shape) if d in src.coords else None
        moved += region_size(need) - (region_size(region_intersect(need, have)) if have else 0)
    return moved


def _gather_dims(shape, src, dst) -> Tuple[int, ...]:
    dims = set()
    for d in dst.device_ids:
        need = dst.region(d, shape)
        have = src.region(d, shape)
        for i, ((n0, n1), (h0, h1)) in enumerate(zip(need, have)):
            if not (h0 <= n0 and n1 <= h1):
                dims.add(i)
    return tuple(sorted(dims))


def _try_all_to_all(shape, src: TileAssignment, dst: TileAssignment):
    """src sharded n-way on dim i (dst unsharded there); dst sharded n-way on dim j (src unsharded)."""
    ts, td = src.tile_shape, dst.tile_shape
    diff = [k for k in range(len(ts)) if ts[k] != td[k]]
    if len(diff) != 2:
        return None
    a, b = diff
    if ts[a] > 1 and td[a] == 1 and ts[b] == 1 and td[b] == ts[a]:
        i, j = a, b
    elif ts[b] > 1 and td[b] == 1 and ts[a] == 1 and td[a] == ts[b]:
        i, j = b, a
    else:
        return None
    if src.num_replicas != dst.num_replicas:
        return None
    groups = src.groups_along([i])
    perms = []
    for g in groups:
        # all members must agree on every other dim between src and dst
        perm = []
        for d in g:
            sc, dc = src.coords[d], dst.coords[d]
            if any(sc[k] != dc[k] for k in range(len(ts)) if k not in (i, j)):
                return None
            perm.append(dc[j])
        if sorted(perm) != list(range(len(g))):
            return None
        perms.append(perm)
    identity = all(p == list(range(len(p))) for p in perms)
    return ReshardPlan("all_to_all", split_dim=j, concat_dim=i, groups=groups,
                       perms=None if identity else perms)


def plan_reshard(shape, src: TileAssignment, dst: TileAssignment) -> ReshardPlan:
    shape = tuple(shape)
    if src == dst:
        return ReshardPlan("noop")
    same_devs = set(src.device_ids) == set(dst.device_ids)
    if same_devs:
        if all(region_contains(src.region(d, shape), dst.region(d, shape)) for d in dst.device_ids):
            return ReshardPlan("slice")
        a2a = _try_all_to_all(shape, src, dst)
        if a2a is not None:
            return a2a
        xbytes = _exchange_bytes(shape, src, dst)
        gdims = _gather_dims(shape, src, dst)
        if gdims:
            mid = src.unshard(gdims)
            if all(region_contains(mid.region(d, shape), dst.region(d, shape)) for d in dst.device_ids):
                gbytes = sum(region_size(mid.region(d, shape)) - region_size(src.region(d, shape))
                             for d in dst.device_ids)
                if gbytes <= xbytes:
                    return ReshardPlan("all_gather", dims=gdims, groups=src.groups_along(gdims), mid=mid)
        if src.tile_shape == dst.tile_shape and src.num_replicas == dst.num_replicas:
            return ReshardPlan("collective_permute", transfers=_exchange_transfers(shape, src, dst))
    return ReshardPlan("exchange", transfers=_exchange_transfers(shape, src, dst))


def reshard_cost(shape, src: TileAssignment, dst: TileAssignment) -> int:
    """Elements moved between devices (the partitioner's cost model)."""
    if src == dst:
        return 0
    if set(src.device_ids) == set(dst.device_ids):
        return _exchange_bytes(tuple(shape), src, dst)
    return sum(region_size(dst.region(d, shape)) for d in dst.device_ids)


def _local_slice(x: ShardedArray, src: TileAssignment, dst: TileAssignment, shape) -> Dict[int, torch.Tensor]:
    out = {}
    for d, t in x.local.items():
        if d not in dst.coords:
            continue
        rel = _rel(dst.region(d, shape), src.region(d, shape))
        if all(r.start == 0 and r.stop == n for r, n in zip(rel, t.shape)):
            out[d] = t
        elif t.is_cuda:
            from ..ops import hip as _hip
            out[d] = _hip.box_slice(t, rel)
        else:
            out[d] = t[rel]
    return out


def reshard_tile(x: ShardedArray, dst: TileAssignment, sharding: Optional[Sharding] = None,
                 note: str = "") -> ShardedArray:
    src = x.tile
    shape = x.shape
    dst.check_shape(shape)
    if sharding is None:
        sharding = sharding_from_tile(dst, like=[x.sharding])
    p = plan_reshard(shape, src, dst)
    k = p.kind
    if k == "noop":
        return ShardedArray(shape, x.dtype, sharding, x.local)
    if k == "slice":
        return ShardedArray(shape, x.dtype, sharding, _local_slice(x, src, dst, shape))
    if k == "all_to_all":
        loc = C.all_to_all(x.local, p.info["groups"], p.info["split_dim"], p.info["concat_dim"],
                           perms=p.info["perms"], note=note)
        return ShardedArray(shape, x.dtype, sharding, loc)
    if k == "all_gather":
        loc = x.local
        cur = src
        for dim in p.info["dims"]:
            groups = cur.groups_along([dim])
            loc = C.all_gather(loc, groups, dim, note=note)
            cur = cur.unshard([dim])
        tmp = ShardedArray(shape, x.dtype, sharding, loc)
        if cur != dst:
            loc = _local_slice(tmp, cur, dst, shape)
        return ShardedArray(shape, x.dtype, sharding, loc)
    # point-to-point exchange / permute
    pi = process_index()
    out_meta = {}
    ss = dst.shard_shape(shape)
    any_local = next(iter(x.local.values())) if x.local else None
    meta = any(t.is_meta for t in x.local.values())
    for d in dst.device_ids:
        dev = get_device(d)
        if dev.process_index != pi:
            continue
        out_meta[d] = (ss, x.dtype, torch.device("meta") if meta else dev.torch_device)
    loc = C.exchange(x.local, p.info["transfers"], out_meta, kind=k, note=note)
    return ShardedArray(shape, x.dtype, sharding, loc)


def reshard(x: ShardedArray, sharding: Sharding) -> ShardedArray:
    dst = sharding.tile_assignment(x.ndim)
    return reshard_tile(x, dst, sharding)
