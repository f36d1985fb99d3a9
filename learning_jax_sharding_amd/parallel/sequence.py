"""Sequence / context parallelism for attention.

The reference shards the sequence over ``model`` through the (misnamed) ``embed`` logical
axis on activations (``case6_attention.py:105-107,114-116,161``) and GSPMD gathers the full
K/V before the score einsum (``case6_attention.py:125-133``; SURVEY §2.7 "AG K", "AG V").
Two schedules are provided on (batch, seq, heads, head_dim) arrays whose seq dim is sharded:

* ``mode="allgather"`` - the reference's plan: all-gather K and V over the sequence group,
  then one flash-attention kernel per shard with its query offset (this is what
  :func:`ops.core.dot_product_attention` lowers to);
* ``mode="ring"`` - ring attention: the K/V blocks travel around the sequence group; each
  step runs the flash kernel of the local queries against the block in hand and merges
  the partial softmax through the log-sum-exp (the kernels' log2 domain), so no device
  ever holds more than two K/V blocks.  The backward replays the ring with the GLOBAL
  log-sum-exp and final output (flash backward is blockwise separable): dQ accumulates
  locally, dK/dV accumulators travel with their blocks and arrive home after the last
  hop.  Causal blocks entirely above the diagonal are skipped.

* ``mode="ulysses"`` - DeepSpeed-Ulysses: ONE all-to-all per tensor moves q, k and v from
  sequence-sharded to head-sharded (every device then holds the full sequence of H/n heads),
  the flash kernel runs locally with no K/V traffic of its own, and one all-to-all brings the
  output back to sequence sharding.  Per device it moves 3 + 1 tensors of (n-1)/n of its shard
  (the all-gather plan receives (n-1) shards of K and V), and the attention kernels see the
  single-device shape (all keys, whole heads) instead of S/n-query blocks against S keys.
  Needs the head count divisible by n; the backward is the transposed all-to-alls.

Memory per device is O(S/n) for K/V instead of O(S), the stepping stone to long-context
training on 288 GB parts; on xGMI the hop is a point-to-point neighbour transfer, one link.
Each hop's K/V transfer is issued on a side HIP stream before the current block's flash
kernel and joined after it, so the transfer overlaps the attention compute.  The
partial softmaxes are merged by log-sum-exp INSIDE the forward kernel's epilogue (running f32
output + lse, ``ops.kernels.attention_fwd_merge``), and in the backward the dK/dV accumulators'
hops run on the side stream while the next block's backward computes.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import torch

from ..array import ShardedArray
from ..comm import collectives as C
from ..comm.backend import Transfer
from ..ops import core
from ..ops import kernels as K
from ..spmd import plan as _plan
from ..spmd.reshard import reshard_tile

__all__ = ["context_parallel_attention", "ring_attention", "ulysses_attention"]


def context_parallel_attention(q: ShardedArray, k: ShardedArray, v: ShardedArray, scale: Optional[float] = None,
                               causal: bool = False, mode: str = "allgather") -> ShardedArray:
    if mode == "allgather":
        return core.dot_product_attention(q, k, v, scale=scale, causal=causal)
    if mode == "ring":
        return ring_attention(q, k, v, scale=scale, causal=causal)
    if mode == "ulysses":
        return ulysses_attention(q, k, v, scale=scale, causal=causal)
    raise ValueError(f"unknown context-parallel mode {mode!r}")


# ----------------------------------------------------------------------------- ulysses
def _seq_to_heads(t):
    """The tile of ``t`` [batch, seq, heads, d] with its sequence split moved onto the heads: the
    device holding sequence block i of a group holds head block i of the full sequence."""
    from ..sharding.tile import TileAssignment
    ts = t.tile_shape
    coords = {d: (c[0], 0, c[1]) + tuple(c[3:]) for d, c in t.coords.items()}
    return TileAssignment.from_coords(coords, (ts[0], 1, ts[1]) + tuple(ts[3:]))


def ulysses_attention(q: ShardedArray, k: ShardedArray, v: ShardedArray, scale: Optional[float] = None,
                      causal: bool = False) -> ShardedArray:
    """All-to-all (sequence <-> heads) attention over q's sequence sharding (see module doc); the
    all-gather plan when the heads are already split or do not divide over the group."""
    if scale is None:
        scale = q.shape[-1] ** -0.5
    qt = q.tile
    if qt.tile_shape[3] > 1:
        q = reshard_tile(q, qt.unshard([3]), note="ulysses.q")
        qt = q.tile
    n = qt.tile_shape[1]
    if n == 1 or qt.tile_shape[2] != 1 or q.shape[2] % n:
        return core.dot_product_attention(q, k, v, scale=scale, causal=causal)
    ht = _seq_to_heads(qt)
    if ht is None:
        return core.dot_product_attention(q, k, v, scale=scale, causal=causal)
    _plan.record("ulysses_attention", group=n, q_tiles=qt.tile_shape, head_tiles=ht.tile_shape)
    qh = reshard_tile(q, ht, note="ulysses.q")
    kh = reshard_tile(k, ht, note="ulysses.k")
    vh = reshard_tile(v, ht, note="ulysses.v")
    oh = core.dot_product_attention(qh, kh, vh, scale=scale, causal=causal)
    return reshard_tile(oh, qt, note="ulysses.out")


# ----------------------------------------------------------------------------- ring
def _full(t: torch.Tensor):
    return tuple(slice(0, s) for s in t.shape)


def _rotate(xs: Dict[int, torch.Tensor], nxt: Dict[int, int]) -> Dict[int, torch.Tensor]:
    """Send every device's tensor to its ring successor (one point-to-point hop).  The
    transfer list is global (every ring member's hop, identical on all processes); each
    process only holds - and receives into - its own devices' blocks."""
    t0 = next(iter(xs.values()))
    full = _full(t0)
    transfers = [Transfer(nxt[d], d, full, full) for d in sorted(nxt)]
    meta = {d: (tuple(t.shape), t.dtype, t.device) for d, t in xs.items()}
    return C._run(C._Spec("exchange", transfers=transfers, out_meta=meta), xs)


_SIDE: Dict[int, "torch.cuda.Stream"] = {}


def _rotate_async(bufs: List[Dict[int, torch.Tensor]], nxt: Dict[int, int]):
    """Start the next ring hop of every dict in ``bufs`` on a side HIP stream per GPU (after the
    current stream's producers), so the hop overlaps the attention block computed meanwhile on
    the compute stream.  Returns a thunk that makes the compute stream wait for the hop and
    hands back the rotated dicts (host devices: the hop simply runs)."""
    import contextlib
    t0 = next(iter(bufs[0].values()))
    from ..spmd import graphs as _graphs
    if not t0.is_cuda or not _graphs.forks_ok():   # (host arrays, or a capture cut at the hops)
        out = [_rotate(b, nxt) for b in bufs]
        return lambda: out
    gpus = sorted({t.device.index for b in bufs for t in b.values()})
    events = []
    for g in gpus:
        side = _SIDE.get(g)
        if side is None:
            side = _SIDE[g] = torch.cuda.Stream(device=g)
        side.wait_stream(torch.cuda.current_stream(g))
    streams = [_SIDE[g] for g in gpus]
    # every GPU's side stream is made current for its device (a single-controller run drives
    # several GPUs from this thread; one rank per GPU has exactly one)
    with contextlib.ExitStack() as es:
        for st in streams:
            es.enter_context(torch.cuda.stream(st))
        out = [_rotate(b, nxt) for b in bufs]
        for g, st in zip(gpus, streams):
            ev = torch.cuda.Event()
            ev.record(st)
            events.append((g, ev))

    def join():
        for g, ev in events:
            cur = torch.cuda.current_stream(g)
            cur.wait_event(ev)
        for b in out:
            for t in b.values():
                t.record_stream(torch.cuda.current_stream(t.device))
        return out
    return join


class _RingAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, meta, devs, *flat):
        scale, causal, pos, n, nxt, prv, s_loc = meta
        nd = len(devs)
        q = dict(zip(devs, flat[:nd]))
        kk = dict(zip(devs, flat[nd:2 * nd]))
        vv = dict(zip(devs, flat[2 * nd:]))
        # the hops each device computes (causal: blocks entirely above the diagonal are skipped);
        # the last one writes the final output
        hops = {d: [s for s in range(n) if not (causal and (pos[d] - s) % n > pos[d])] for d in devs}
        state = {d: [None, None] for d in devs}            # running (O f32, lse), merged in-kernel
        out = {}
        kb, vb = dict(kk), dict(vv)
        for s in range(n):
            # hop s+1's K/V transfer runs on the side stream while block s computes
            pending = _rotate_async([kb, vb], nxt) if s + 1 < n else None
            for d in devs:
                if s not in hops[d]:
                    continue
                j = (pos[d] - s) % n                       # global block index of the kv in hand
                r = K.attention_fwd_merge(q[d], kb[d], vb[d], scale, causal, (pos[d] - j) * s_loc, state[d],
                                          last=s == hops[d][-1])
                if r is not None:
                    out[d] = r
            if pending is not None:
                kb, vb = pending()
        outs = [out[d] for d in devs]
        ctx.meta = meta
        ctx.devs = devs
        ctx.hops = hops
        ctx.save_for_backward(*flat, *outs, *[state[d][1] for d in devs])
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gos):
        scale, causal, pos, n, nxt, prv, s_loc = ctx.meta
        devs, hops = ctx.devs, ctx.hops
        nd = len(devs)
        saved = ctx.saved_tensors
        q = dict(zip(devs, saved[:nd]))
        kb = dict(zip(devs, saved[nd:2 * nd]))
        vb = dict(zip(devs, saved[2 * nd:3 * nd]))
        o = dict(zip(devs, saved[3 * nd:4 * nd]))
        lse = dict(zip(devs, saved[4 * nd:5 * nd]))
        do = {d: (g if g is not None else torch.zeros_like(o[d])) for d, g in zip(devs, gos)}
        dq = {d: None for d in devs}
        acc = None                 # join thunk of the dK/dV accumulators in flight
        for s in range(n):
            # the next K/V blocks travel on the side stream during this block's backward
            pending = _rotate_async([kb, vb], nxt) if s + 1 < n else None
            contrib = {}
            for d in devs:
                if s not in hops[d]:
                    continue
                j = (pos[d] - s) % n
                gq, gk, gv = K.attention_bwd_block(q[d], kb[d], vb[d], o[d], do[d], lse[d], scale, causal,
                                                   (pos[d] - j) * s_loc)
                dq[d] = gq.float() if dq[d] is None else dq[d].add_(gq)
                contrib[d] = (gk, gv)
            # the dK/dV accumulators travel with their kv blocks; each hop is started as soon as
            # this block has added to them and lands while the NEXT block computes (only the add
            # waits for it); n hops bring every accumulator home
            if acc is None:
                dk = {d: (contrib[d][0].float() if d in contrib else torch.zeros(kb[d].shape, dtype=torch.float32,
                                                                                 device=kb[d].device)) for d in devs}
                dv = {d: (contrib[d][1].float() if d in contrib else torch.zeros(vb[d].shape, dtype=torch.float32,
                                                                                 device=vb[d].device)) for d in devs}
            else:
                dk, dv = acc()
                for d, (gk, gv) in contrib.items():
                    dk[d].add_(gk)
                    dv[d].add_(gv)
            acc = _rotate_async([dk, dv], nxt)
            if pending is not None:
                kb, vb = pending()
        dk, dv = acc()
        grads = [(dq[d] if dq[d] is not None else torch.zeros_like(q[d], dtype=torch.float32)).to(q[d].dtype)
                 for d in devs] + [dk[d].to(kb[d].dtype) for d in devs] + [dv[d].to(vb[d].dtype) for d in devs]
        return (None, None) + tuple(grads)


def ring_attention(q: ShardedArray, k: ShardedArray, v: ShardedArray, scale: Optional[float] = None,
                   causal: bool = False) -> ShardedArray:
    """Ring (blockwise, log-sum-exp merged) attention over q's sequence sharding."""
    if scale is None:
        scale = q.shape[-1] ** -0.5
    qt = q.tile
    if qt.tile_shape[3] > 1:
        q = reshard_tile(q, qt.unshard([3]), note="ring.q")
        qt = q.tile
    k = reshard_tile(k, qt, note="ring.k") if k.tile != qt else k
    v = reshard_tile(v, qt, note="ring.v") if v.tile != qt else v
    n = qt.tile_shape[1]
    if n == 1:
        return core.dot_product_attention(q, k, v, scale=scale, causal=causal)
    groups = qt.groups_along([1])
    pos, nxt, prv = {}, {}, {}
    for g in groups:
        for i, d in enumerate(g):
            pos[d] = i
            nxt[d] = g[(i + 1) % len(g)]
            prv[d] = g[(i - 1) % len(g)]
    s_loc = qt.shard_shape(q.shape)[1]
    devs = tuple(sorted(q.local))
    _plan.record("ring_attention", ring=n, q_tiles=qt.tile_shape, hops=n - 1)
    meta = (float(scale), bool(causal), pos, n, nxt, prv, s_loc)
    flat = [q.local[d] for d in devs] + [k.local[d] for d in devs] + [v.local[d] for d in devs]
    outs = _RingAttention.apply(meta, devs, *flat)
    return ShardedArray(q.shape, v.dtype, q.sharding, dict(zip(devs, outs)))
