"""Differentiable collectives over device groups.

Each collective is a ``torch.autograd.Function`` whose backward is the
transposed collective, under the SPMD cotangent convention used throughout the
framework: *the true cotangent of a tile is the sum of the per-device
cotangents over every device holding a copy of that tile*.  Under that
convention (valid because backward passes are linear in the cotangent):

====================  ==============================
forward               backward
====================  ==============================
all_gather(dim)       reduce_scatter(dim)
reduce_scatter(dim)   all_gather(dim)
all_reduce            all_reduce
all_to_all(i -> j)    all_to_all(j -> i)
exchange (gather)     exchange reversed, accumulating
====================  ==============================

This is the "collectives transpose: AG<->RS, A2A<->A2A" requirement of
SURVEY §3.3, realised on torch autograd instead of a separate AD system.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..spmd import plan as _plan
from .backend import Transfer, get_comm

__all__ = ["all_gather", "reduce_scatter", "all_reduce", "all_to_all", "exchange"]


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


class _Spec:
    __slots__ = ("kind", "groups", "dim", "split_dim", "concat_dim", "perms", "transfers", "out_meta",
                 "accumulate", "reorder")

    def __init__(self, kind, groups=None, dim=None, split_dim=None, concat_dim=None, perms=None,
                 transfers=None, out_meta=None, accumulate=False, reorder=None):
        self.kind = kind
        self.groups = groups
        self.dim = dim
        self.split_dim = split_dim
        self.concat_dim = concat_dim
        self.perms = perms
        self.transfers = transfers
        self.out_meta = out_meta
        self.accumulate = accumulate
        self.reorder = reorder


def _group_size(spec: _Spec, d: int) -> int:
    return next(len(g) for g in spec.groups if d in g)


def _run_meta(spec: _Spec, xs: Dict[int, torch.Tensor]) -> Dict[int, torch.Tensor]:
    """Abstract evaluation (``eval_shape`` on meta tensors): output shapes only, no traffic -
    a process-group backend cannot run collectives on meta tensors, and must not try."""
    k = spec.kind
    out = {}
    if k == "exchange":
        from ..runtime.devices import local_devices
        mine = {dv.id for dv in local_devices()}
        return {d: torch.empty(shape, dtype=dt, device="meta") for d, (shape, dt, _) in spec.out_meta.items()
                if d in mine or d in xs}
    for d, x in xs.items():
        shp = list(x.shape)
        n = _group_size(spec, d)
        if k == "all_gather":
            shp[spec.dim] *= n
        elif k == "reduce_scatter":
            shp[spec.dim] //= n
        elif k == "all_to_all":
            shp[spec.split_dim] //= n
            shp[spec.concat_dim] *= n
        out[d] = torch.empty(shp, dtype=x.dtype, device="meta")
    return out


def _run(spec: _Spec, xs: Dict[int, torch.Tensor]) -> Dict[int, torch.Tensor]:
    if any(t.device.type == "meta" for t in xs.values()):
        return _run_meta(spec, xs)
    comm = get_comm()
    out = None
    if comm.kind == "dist" and any(t.is_cuda for t in xs.values()):
        # cross-process collectives through torch process groups are cut points of a segmented
        # HIP-graph capture; native RCCL ones are captured like kernels
        from ..spmd import graphs
        x0 = next(iter(xs.values()))
        if graphs.current() is not None and not comm.graph_safe(spec.kind, x0, spec.groups):
            out = graphs.run_collective(lambda: _run_local(comm, spec, xs),
                                        what=f"{spec.kind} {tuple(x0.shape)} {x0.dtype}")[0]
    if out is None:
        out = _run_local(comm, spec, xs)
    if _DEBUG:
        from ..profiler import after_collective
        after_collective(spec.kind, out)
    return out


_DEBUG = os.environ.get("LJS_DEBUG_SYNC", "0") == "1" or os.environ.get("LJS_DEBUG_NANS", "0") == "1"


def _run_local(comm, spec: _Spec, xs: Dict[int, torch.Tensor]) -> Dict[int, torch.Tensor]:
    k = spec.kind
    if k == "all_gather":
        return comm.all_gather(xs, spec.groups, spec.dim)
    if k == "reduce_scatter":
        return comm.reduce_scatter(xs, spec.groups, spec.dim)
    if k == "all_reduce":
        return comm.all_reduce(xs, spec.groups)
    if k == "all_to_all":
        out = comm.all_to_all(xs, spec.groups, spec.split_dim, spec.concat_dim, spec.perms)
        if spec.reorder is not None:
            # member j's output chunk p (along concat_dim) must come from the member i with perm_i = p
            res = {}
            for gi, g in enumerate(spec.groups):
                inv = spec.reorder[gi]
                for d in g:
                    if d in out:
                        ch = out[d].chunk(len(g), spec.concat_dim)
                        res[d] = torch.cat([ch[i] for i in inv], spec.concat_dim).contiguous()
            return res
        return out
    if k == "exchange":
        return comm.exchange(xs, spec.transfers, spec.out_meta, spec.accumulate)
    raise ValueError(k)


def _transpose(spec: _Spec, in_meta) -> _Spec:
    k = spec.kind
    if k == "all_gather":
        return _Spec("reduce_scatter", spec.groups, dim=spec.dim)
    if k == "reduce_scatter":
        return _Spec("all_gather", spec.groups, dim=spec.dim)
    if k == "all_reduce":
        return _Spec("all_reduce", spec.groups)
    if k == "all_to_all":
        reorder = None
        if spec.perms is not None:
            # forward: receiver i takes chunk perm[i] of each sender.  Backward: sender-side chunk j
            # of receiver i's gradient goes back to member j at split position perm[i].
            reorder = []
            for perm in spec.perms:
                inv = [0] * len(perm)
                for i, p in enumerate(perm):
                    inv[p] = i
                reorder.append(inv)
        return _Spec("all_to_all", spec.groups, split_dim=spec.concat_dim, concat_dim=spec.split_dim,
                     reorder=reorder)
    if k == "exchange":
        return _Spec("exchange", transfers=[t.reversed() for t in spec.transfers], out_meta=in_meta,
                     accumulate=True)
    raise ValueError(k)


class _CollectiveFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec, in_devs, out_devs, *xs):
        ctx.spec = spec
        ctx.in_devs = in_devs
        ctx.out_devs = out_devs
        ctx.in_meta = {d: (tuple(x.shape), x.dtype, x.device) for d, x in zip(in_devs, xs)}
        # a pure permutation of elements over the devices: keep the inputs' METADATA so a constant
        # cotangent on every output can be moved to them without running the transpose
        # (spmd.api.value_and_grad: the seed of a summed loss; the sum is permutation-invariant).
        # Not the tensors - an activation held to the backward would only cost memory: the seed
        # goes to the inputs' gradient edges (this node's next_functions)
        ctx.perm_inputs = tuple((tuple(x.shape), x.dtype, x.device, x.requires_grad) for x in xs) \
            if spec.kind == "all_to_all" and tuple(in_devs) == tuple(out_devs) else None
        out = _run(spec, dict(zip(in_devs, xs)))
        ctx.out_meta = {d: (tuple(out[d].shape), out[d].dtype, out[d].device) for d in out_devs}
        ctx.out_strides = {d: tuple(out[d].stride()) for d in out_devs}
        return tuple(out[d] for d in out_devs)

    @staticmethod
    def backward(ctx, *gs):
        gd = {}
        from ..ops.hip import is_dense
        for d, g in zip(ctx.out_devs, gs):
            if g is None:
                shape, dt, dev = ctx.out_meta[d]
                g = torch.zeros(shape, dtype=dt, device=dev)
            elif not is_dense(g):
                # materialise in the forward output's layout (a seq-major output's gradient then
                # moves back over the sequence as contiguous blocks)
                shape, dt, dev = ctx.out_meta[d]
                st = ctx.out_strides[d]
                buf = torch.empty_strided(shape, st, dtype=g.dtype, device=dev) if _dense_strides(shape, st) \
                    else torch.empty(shape, dtype=g.dtype, device=dev)
                g = buf.copy_(g)
            gd[d] = g
        tspec = _transpose(ctx.spec, ctx.in_meta)
        kind = "collective_permute" if tspec.kind == "exchange" else tspec.kind
        _plan.record(kind, groups=tspec.groups, note="backward", bytes_in=_per_device_bytes(gd))
        out = _run(tspec, gd)
        return (None, None, None) + tuple(out.get(d) for d in ctx.in_devs)


def _dense_strides(shape, strides) -> bool:
    dims = sorted((i for i in range(len(shape)) if shape[i] > 1), key=lambda i: -strides[i])
    exp = 1
    for i in reversed(dims):
        if strides[i] != exp:
            return False
        exp *= shape[i]
    return True


def _apply(spec: _Spec, xs: Dict[int, torch.Tensor], out_devs: Optional[Sequence[int]] = None):
    in_devs = tuple(sorted(xs))
    out_devs = tuple(sorted(out_devs)) if out_devs is not None else in_devs
    ts = [xs[d] for d in in_devs]
    if torch.is_grad_enabled() and any(t.requires_grad for t in ts):
        outs = _CollectiveFn.apply(spec, in_devs, out_devs, *ts)
        return dict(zip(out_devs, outs))
    out = _run(spec, dict(zip(in_devs, ts)))
    return {d: out[d] for d in out_devs}


def _per_device_bytes(xs: Dict[int, torch.Tensor]) -> int:
    return max((_nbytes(t) for t in xs.values()), default=0)


def all_gather(xs, groups, dim: int, **note):
    _plan.record("all_gather", dim=dim, groups=tuple(tuple(g) for g in groups),
                 bytes_in=_per_device_bytes(xs), **note)
    return _apply(_Spec("all_gather", groups, dim=dim), xs)


def reduce_scatter(xs, groups, dim: int, **note):
    _plan.record("reduce_scatter", dim=dim, groups=tuple(tuple(g) for g in groups),
                 bytes_in=_per_device_bytes(xs), **note)
    return _apply(_Spec("reduce_scatter", groups, dim=dim), xs)


def all_reduce(xs, groups, **note):
    groups = [tuple(g) for g in groups]
    if all(len(g) == 1 for g in groups):
        return dict(xs)
    _plan.record("all_reduce", groups=tuple(groups), bytes_in=_per_device_bytes(xs), **note)
    return _apply(_Spec("all_reduce", groups), xs)


def all_to_all(xs, groups, split_dim: int, concat_dim: int, perms=None, **note):
    _plan.record("all_to_all", split_dim=split_dim, concat_dim=concat_dim,
                 groups=tuple(tuple(g) for g in groups), bytes_in=_per_device_bytes(xs), **note)
    return _apply(_Spec("all_to_all", groups, split_dim=split_dim, concat_dim=concat_dim, perms=perms), xs)


def exchange(xs, transfers: Sequence[Transfer], out_meta, kind: str = "exchange", **note):
    moved = [t for t in transfers if t.src != t.dst]
    if moved:
        _plan.record(kind, n_transfers=len(moved), transfers=list(moved),
                     bytes_moved=None, **note)
    return _apply(_Spec("exchange", transfers=list(transfers), out_meta=dict(out_meta)), xs,
                  out_devs=list(out_meta))
