"""All-gather of sharded weights as their bf16 GEMM shadows.

When a layer's f32 weight is sharded and its GEMM needs it whole - FSDP's gather at use
(``case5_attention_dense.py:109-112``, ``case3_fully_sharded.py:23-46,57``) or the reference's
Q/K/V weights sharded over ``model`` (``case6_attention.py:56-59,183-187``) - the partitioner's
generic plan gathers the f32 master shards and every step then casts + transposes the gathered
copy for the MFMA GEMM.  But each shard already HAS its bf16 transposed shadow, rewritten by the
fused Adam in the pass that updates it (``ops/shadow.py``).  Gathering those instead:

* moves half the bytes over xGMI (bf16, not f32);
* needs no cast kernel on the gathered weight;
* stacks Q/K/V: one collective of the three shards' stacked shadows ``[3][N][K/n]`` and one
  unpack into the ``[3][N][K]`` operand of the batched QKV GEMM.

The gathered weight is handed to the layer as an f32 PROXY - an uninitialised tensor of the full
shape whose shadow registry entry points at the gathered bf16 copy (``shadow.register_proxy``):
the GEMMs read the bf16 copy; the backward's plain ``[in][out]`` shadow is transposed from it;
nothing may read the proxy's f32 values (the registry raises).  The proxy is the output of a
differentiable gather whose backward is the reduce-scatter of the full f32 gradient onto the
shards - the transposed collective, as for the generic all-gather.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import torch

from ..array import ShardedArray
from ..comm import collectives as C
from ..sharding.shardings import sharding_from_tile
from ..sharding.tile import TileAssignment
from ..spmd import plan as _plan

__all__ = ["eligible", "gather_bf16", "mx_eligible", "gather_mx"]

_ON = os.environ.get("LJS_GATHER_SHADOWS", "1") == "1"
# how the backward reduce-scatters ran (tests / diagnostics): one-pass slab sums vs combined grads
STATS = {"slab_sum": 0, "combined": 0, "stacked": 0}


def _gather_dim(src: TileAssignment, dst: TileAssignment, shape) -> Optional[int]:
    """The one dim along which ``dst`` is ``src`` all-gathered (no slicing, no permutation)."""
    from ..spmd.reshard import plan_reshard
    p = plan_reshard(tuple(shape), src, dst)
    if p.kind != "all_gather" or len(p.info["dims"]) != 1:
        return None
    dim = p.info["dims"][0]
    return dim if src.unshard([dim]) == dst else None


def eligible(kernels: Sequence[ShardedArray], dst: TileAssignment) -> Optional[int]:
    """Gather dim when every kernel is a 2-D f32 GPU weight that ``dst`` all-gathers along one dim."""
    if not _ON or not kernels:
        return None
    k0 = kernels[0]
    if k0.ndim != 2 or k0.dtype != torch.float32 or k0.tile == dst:
        return None
    for k in kernels:
        if k.tile != k0.tile or tuple(k.shape) != tuple(k0.shape) or k.dtype != torch.float32:
            return None
        if not k.local or not all(t.is_cuda and t.is_contiguous() for t in k.local.values()):
            return None
    dim = _gather_dim(k0.tile, dst, k0.shape)
    if dim is None:
        return None
    n = k0.tile.tile_shape[dim]
    K, N = k0.shape
    # the shards' shadows: "T" = [N][K_loc] for dim 0 (gather along its columns), [N_loc][K] for dim 1
    if (K if dim == 0 else N) % n or (K // n if dim == 0 else N // n) % 8:
        return None
    return dim


def _loopback(groups, xs) -> bool:
    """Every group's members are virtual devices of ONE GPU under the single-process backend (the
    collective is a local copy / sum, no RCCL)."""
    from ..comm.backend import get_comm
    if get_comm().kind != "local":
        return False
    for g in groups:
        ts = [xs.get(d) for d in g]
        if any(t is None for t in ts) or not ts[0].is_cuda or any(t.device != ts[0].device for t in ts):
            return False
    return True


def _slab_sum(groups, dim, devs, ents, shape):
    """Loopback reduce-scatter of uncombined weight gradients: per group, ONE pass sums every
    member's split-K slabs (hip.SlabGrad, contiguous [K][N] each) into the full gradient, whose
    chunks along ``dim`` are the members' shards - no per-device slab combine, no second sum."""
    from ..ops import hip
    out = {}
    for g in groups:
        ptrs = []
        for d in g:
            sg = ents[d][0]
            base = sg.slabs.data_ptr() + 4 * sg.offset
            ptrs += [base + 4 * s * sg.slab_stride for s in range(sg.S)]
        total = torch.empty(shape, dtype=torch.float32, device=ents[g[0]][0].slabs.device)
        hip.sum_ptrs(ptrs, total)
        for i, ch in enumerate(total.chunk(len(g), dim)):
            out[g[i]] = hip.dense(ch)
    return out


def _slabs_ok(ents, devs, shape) -> bool:
    if len(ents) != len(devs):
        return False
    sgs = [ents[d][0] for d in devs]
    return (all(isinstance(sg, _hip_cls("SlabGrad")) for sg in sgs) and all(
        tuple(sg.shape) == tuple(shape) and sg.ld == shape[1] and sg.slabs.dtype == torch.float32
        and (sg.slabs.data_ptr() + 4 * sg.offset) % 16 == 0 and (4 * sg.slab_stride) % 16 == 0 for sg in sgs)
        and sum(sg.S for sg in sgs) <= 128)


def _stacked_grads(gs, devs, nw, pend):
    """{device: [nw][K][N] view} when every device's nw gradients are consecutive [K][N] slices of
    one f32 buffer and none is still uncombined (``pend``); else None."""
    if nw < 2:
        return None
    out = {}
    for j, d in enumerate(devs):
        g0 = gs[j * nw]
        if g0 is None or g0.dtype != torch.float32 or not g0.is_contiguous() or g0.dim() != 2:
            return None
        K, N = g0.shape
        st = g0.untyped_storage()
        for i in range(nw):
            g = gs[j * nw + i]
            if (g is None or not g.is_contiguous() or tuple(g.shape) != (K, N) or g.dtype != g0.dtype
                    or g.untyped_storage().data_ptr() != st.data_ptr()
                    or g.data_ptr() != g0.data_ptr() + i * K * N * 4
                    or (pend is not None and g.data_ptr() in pend)):
                return None
        if (g0.storage_offset() + nw * K * N) * 4 > st.nbytes():
            return None
        out[d] = torch.as_strided(g0, (nw, K, N), (K * N, N, 1))
    return out


def _hip_cls(name):
    from ..ops import hip
    return getattr(hip, name)


class _GatherBf16(torch.autograd.Function):
    """All local devices at once (a loopback group holds several): f32 shards -> f32 proxies of
    the gathered weights (the forward moves the shards' bf16 shadows); backward reduce-scatters
    the proxies' f32 gradients onto the shards."""

    @staticmethod
    def forward(ctx, meta, *flat):
        groups, dim, devs, nw, n = meta
        from ..ops import hip, shadow
        t_loc = {}
        for j, d in enumerate(devs):
            ws = list(flat[j * nw:(j + 1) * nw])
            # [nw][N_loc][K_loc] shadows in ONE buffer (the fused Adam keeps them there)
            t_loc[d] = shadow.get(ws[0], "T").unsqueeze(0) if nw == 1 else shadow.get_stacked(ws)
        # gather along the shadow's K axis (dim 0 of W) or its N axis (dim 1 of W)
        gdim = 2 if dim == 0 else 1
        if _loopback(groups, t_loc):
            # virtual devices of one GPU: ONE concatenation per group, shared by its members
            # (the proxies are read-only stand-ins; nothing writes the gathered shadow)
            gathered = {}
            for grp in groups:
                buf = hip.concat_parts([t_loc[d] for d in grp], gdim)
                for d in grp:
                    gathered[d] = buf
        else:
            gathered = C._run(C._Spec("all_gather", groups, dim=gdim), t_loc)
        K_loc, N_loc = flat[0].shape
        K, N = (K_loc * n, N_loc) if dim == 0 else (K_loc, N_loc * n)
        outs = []
        dense = {}
        holders = {}
        for j, d in enumerate(devs):
            g = gathered[d]
            if id(g) not in dense:
                dense[id(g)] = g if g.is_contiguous() else g.contiguous()   # [nw][N][K] bf16
            gid, g = id(g), dense[id(g)]
            for i in range(nw):
                p = torch.empty((K, N), dtype=torch.float32, device=flat[j * nw].device)
                shadow.register_proxy(p, g[i], shared=holders.setdefault((gid, i), {}))
                outs.append(p)
        ctx.meta = meta
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        groups, dim, devs, nw, n = ctx.meta
        _plan.record("reduce_scatter", groups=groups, note="backward.bf16_shadow_gather")
        from ..ops import linear as _lin
        res = [None] * len(gs)
        pend = _lin.deferred_pending()
        stacked = _stacked_grads(gs, devs, nw, pend)
        if stacked is not None and not _loopback(groups, stacked):
            # the nw gradients are slices of one [nw][K][N] buffer on every device (a batched
            # weight-gradient launch): ONE reduce-scatter of the stack, whose shards are slices of
            # one buffer in turn (a gradient bucket takes them without concatenating)
            STATS["stacked"] += 1
            red = C._run(C._Spec("reduce_scatter", groups, dim=dim + 1), stacked)
            for j, d in enumerate(devs):
                for i in range(nw):
                    res[j * nw + i] = red[d][i]
            return (None,) + tuple(res)
        for i in range(nw):
            xs, ents = {}, {}
            for j, d in enumerate(devs):
                g = gs[j * nw + i]
                if g is not None:
                    ent = pend.pop(g.data_ptr(), None) if pend is not None else None
                    if ent is not None:
                        ents[d] = ent
                    xs[d] = g
            if ents and len(xs) == len(devs) and _loopback(groups, xs) and _slabs_ok(ents, devs, xs[devs[0]].shape):
                red = _slab_sum(groups, dim, devs, ents, tuple(xs[devs[0]].shape))
                STATS["slab_sum"] += 1
                for j, d in enumerate(devs):
                    res[j * nw + i] = red[d]
                continue
            for ent in ents.values():
                ent[1]()                                   # combine the slabs the usual way
            STATS["combined"] += 1
            xs = {d: g.contiguous() for d, g in xs.items()}
            if len(xs) != len(devs):
                continue
            red = C._run(C._Spec("reduce_scatter", groups, dim=dim), xs)
            for j, d in enumerate(devs):
                res[j * nw + i] = red[d]
        return (None,) + tuple(res)


def gather_bf16(kernels: Sequence[ShardedArray], dst: TileAssignment, dim: int, note: str = "") -> List[ShardedArray]:
    """The kernels all-gathered along ``dim`` to ``dst`` as bf16-shadow proxies (see module doc)."""
    k0 = kernels[0]
    src = k0.tile
    groups = src.groups_along([dim])
    n = src.tile_shape[dim]
    _plan.record("all_gather", dim=dim, groups=tuple(tuple(g) for g in groups),
                 bytes_in=sum(next(iter(k.local.values())).numel() * 2 for k in kernels),
                 note=f"{note}.bf16_shadows", dtype="bfloat16", n_weights=len(kernels))
    sh = sharding_from_tile(dst, like=[k0.sharding])
    devs = tuple(sorted(k0.local))
    nw = len(kernels)
    flat = [k.local[d] for d in devs for k in kernels]
    outs = _GatherBf16.apply((tuple(tuple(g) for g in groups), dim, devs, nw, n), *flat)
    return [ShardedArray(k.shape, k.dtype, sh, {d: outs[j * nw + i] for j, d in enumerate(devs)})
            for i, k in enumerate(kernels)]


# ----------------------------------------------------------------------------- MX-fp8 shadow gather
def mx_eligible(w: ShardedArray, dst: TileAssignment) -> Optional[int]:
    """Gather dim when the f32 weight ``w`` (2-D, GPU shards) is all-gathered to ``dst`` along one
    dim and every shard keeps MX-fp8 shadows (``shadow.mx_eligible``: 64-aligned shard shape, so
    no 32-element MX block straddles a shard boundary); else None."""
    if not _ON or w.ndim != 2 or w.dtype != torch.float32 or w.tile == dst or not w.local:
        return None
    from ..ops import shadow
    if not all(t.is_cuda and shadow.mx_eligible(t) for t in w.local.values()):
        return None
    return _gather_dim(w.tile, dst, w.shape)


class _GatherMx(torch.autograd.Function):
    """f32 shards -> f32 proxies of the gathered weight whose MX-fp8 shadows are the shards' own,
    all-gathered: for W [R][C] gathered along dim g, "QN" (codes [R][C], scales [R][C/32]: blocks
    along C) is gathered along g and "QT" (codes [C][R], scales [C][R/32]: blocks along R) along
    1 - g -- both exactly the full weight's MX quantization, since the 64-aligned shards hold whole
    blocks.  A quarter of the f32 gather's bytes, and no per-step quantization of the gathered
    weight.  The backward is the bf16-shadow gather's: the f32 gradient reduce-scattered."""

    @staticmethod
    def forward(ctx, meta, *flat):
        groups, dim, devs, nw, n = meta
        from ..ops import hip, shadow
        parts = {}
        for kind, gd in (("QN", dim), ("QT", 1 - dim)):
            for j in (0, 1):   # codes, scales
                loc = {d: shadow.get_mx(flat[i], kind)[j] for i, d in enumerate(devs)}
                if _loopback(groups, loc):
                    out = {}
                    for grp in groups:
                        buf = hip.concat_parts([loc[d] for d in grp], gd)
                        for d in grp:
                            out[d] = buf
                else:
                    out = C._run(C._Spec("all_gather", groups, dim=gd), loc)
                parts[(kind, j)] = {d: (t if t.is_contiguous() else t.contiguous()) for d, t in out.items()}
        R_loc, C_loc = flat[0].shape
        R, Cn = (R_loc * n, C_loc) if dim == 0 else (R_loc, C_loc * n)
        outs = []
        for d, t in zip(devs, flat):
            # (a dense, uninitialised stand-in: the allocation moves no bytes.  A zero-stride proxy
            # - one element expanded - was tried and failed the 2x2 MX-gather parity test
            # (tests/test_gpu_e2e.py::test_fp8_ff_block_2d_gathers_mx_shadows, gpurun_out/r5a):
            # the FF block's layout checks treat a non-contiguous weight as one to copy, and the
            # copy is not a registered proxy)
            p = torch.empty((R, Cn), dtype=torch.float32, device=t.device)
            shadow.register_mx_proxy(p, {k: (parts[(k, 0)][d], parts[(k, 1)][d]) for k in ("QN", "QT")})
            outs.append(p)
        ctx.meta = meta
        return tuple(outs)

    backward = staticmethod(_GatherBf16.backward)


def gather_mx(w: ShardedArray, dst: TileAssignment, dim: int, note: str = "") -> ShardedArray:
    """``w`` all-gathered along ``dim`` to ``dst`` as an MX-fp8-shadow proxy (see _GatherMx)."""
    src = w.tile
    groups = src.groups_along([dim])
    n = src.tile_shape[dim]
    t0 = next(iter(w.local.values()))
    _plan.record("all_gather", dim=dim, groups=tuple(tuple(g) for g in groups),
                 bytes_in=2 * t0.numel() + 2 * (t0.numel() // 32), note=f"{note}.mx_shadows", dtype="float8_e4m3fn")
    devs = tuple(sorted(w.local))
    outs = _GatherMx.apply((tuple(tuple(g) for g in groups), dim, devs, 1, n), *[w.local[d] for d in devs])
    return ShardedArray(w.shape, w.dtype, sharding_from_tile(dst, like=[w.sharding]),
                        {d: outs[j] for j, d in enumerate(devs)})
