"""Fused dense layer on the MFMA GEMM: ``ys[i] = x @ W_i (+ b) (relu)``.

Forward: one batched GEMM launch over the stacked kernels (Q/K/V share x), reading each
f32 weight through its persistent bf16 transposed shadow (:mod:`.shadow`; refreshed by the
fused Adam kernel, so no per-step cast).  Output columns of the kernels are interleaved in
one ``[M, n*N]`` buffer, so downstream slices (the attention's q/k/v) are views.

Backward:
* ``dX = sum_i dY_i W_i^T``    - (KC, KC) GEMM against the plain bf16 shadow of W_i
  (f32 accumulation across kernels);
* ``dW_i = X^T dY_i``          - both operands read in their natural row-major layout
  through the transposing LDS read (MN-contiguous operands), split-K with f32 atomics; when
  the dY_i are column blocks of one buffer (the attention backward writes dq/dk/dv into one
  ``[M, 3N]`` buffer) all of them go in ONE batched launch;
* ``db = colsum(dY)``.
Gradients that are a broadcast row (the cotangent of ``y.sum()``) are consumed with a zero
leading dimension instead of being materialised.

Epilogue fusions (``hip.gemm``'s operand R):
* ``residual``: ``y = dense(x) + residual`` in the forward GEMM's epilogue (the transformer
  layer's skip connections; bit-exact with the separate bf16 add), gradient passed through;
* ReLU backward in the dX GEMM: when a dense's input is the output of a ReLU dense (recorded
  in the forward), its dX GEMM writes ``dX * (x > 0)`` directly and marks the result, and the
  ReLU dense's backward then skips its own mask pass (masking is idempotent, so a gradient
  that was summed with other contributions on the way is simply masked again).
"""
from __future__ import annotations

import contextlib
import os
import threading
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import hip
from . import shadow

__all__ = ["linear"]

import weakref

# bf16 outputs of ReLU denses (data_ptr -> (weakref, version)) and dX gradients already masked by
# such an output (data_ptr -> (weakref, version, mask data_ptr))
_RELU_OUT = {}
_PREMASKED = {}


def _register(table, t: torch.Tensor, *extra) -> None:
    key = t.data_ptr()
    ref = weakref.ref(t, lambda _r, k=key, tb=table: tb.pop(k, None) if tb.get(k, (None,))[0] is _r else None)
    table[key] = (ref, t._version) + extra


def _lookup(table, t: torch.Tensor):
    ent = table.get(t.data_ptr())
    if ent is None:
        return None
    y = ent[0]()
    if y is None or y._version != ent[1] or y.data_ptr() != t.data_ptr() or y.numel() != t.numel():
        return None
    return ent


def _is_relu_out(t: torch.Tensor) -> bool:
    return _lookup(_RELU_OUT, t) is not None


def _relu_node(x: torch.Tensor) -> bool:
    """Whether ``x`` is an output of a ReLU :class:`_Linear` in the autograd graph (its grad_fn
    is that Function's backward node, whose ctx carries ``meta`` with relu=True)."""
    meta = getattr(x.grad_fn, "meta", None) if x.grad_fn is not None else None
    return bool(meta is not None and len(meta) > 5 and meta[5])


def _premasked_by(dy: torch.Tensor, y: torch.Tensor) -> bool:
    ent = _lookup(_PREMASKED, dy)
    return ent is not None and ent[2] == y.data_ptr() and dy.is_contiguous()


def _splitk(M: int, N: int, K: int, batch: int, tile: int) -> int:
    tiles = -(-M // tile) * -(-N // tile) * batch
    if tiles >= 200:
        return 1
    s = max(1, min(16, round(400 / tiles), K // 1024))
    return s


_DW_SPLIT = 0   # (tests: force the K-chunk count)

# The attention that follows a fused Q/K/V projection (models/attention.py announces it): the
# projection then runs hip.qkv_attn_fwd -- the GEMM and each (batch, head)'s attention forward in
# one kernel -- and leaves (o, lse) for the attention op (hip._take_fused_attention).
# LJS_QKV_ATTN=0: the GEMM alone (the attention runs its own kernel).
_QKV_ATTN = os.environ.get("LJS_QKV_ATTN", "1") != "0"
_ATTN_NEXT: List[Optional[tuple]] = [None]


@contextlib.contextmanager
def attention_next(heads: int, dim_head: int, scale: float):
    """Inside: a 3-weight dense whose outputs are the q / k / v of a non-causal self-attention
    with ``heads`` x ``dim_head`` heads and softmax ``scale`` (fused when the shapes allow)."""
    prev = _ATTN_NEXT[0]
    _ATTN_NEXT[0] = (int(heads), int(dim_head), float(scale)) if _QKV_ATTN else None
    try:
        yield
    finally:
        _ATTN_NEXT[0] = prev


def _fuse_attention_ok(x, xb, wt, nw, N, K, b, relu, res, od, out_dtype, wmajor, order, swap) -> Optional[tuple]:
    fz = _ATTN_NEXT[0]
    if fz is None or nw != 3 or b is not None or relu or res is not None or swap or wmajor:
        return None
    heads, dh, _ = fz
    if not (od == torch.bfloat16 and out_dtype == torch.bfloat16 and x.is_cuda and x.dim() == 3
            and order == (0, 1, 2) and x.shape[1] == 256 and dh == 64 and N == heads * 64 and K % 128 == 0
            and xb.dtype == torch.bfloat16 and xb.stride(1) == 1 and xb.stride(0) % 8 == 0
            and xb.data_ptr() % 16 == 0 and wt.is_contiguous() and wt.data_ptr() % 16 == 0):
        return None
    # one 8-wave block per CU over (batch, head) items: with fewer items than half the CUs the
    # fused kernel leaves CUs idle that the separate GEMM + attention fill (B = 8, 64 items: step
    # 0.0796 vs 0.0732 ms, gpurun_out/r6g); from half the CUs up it wins (B = 16, 128 items:
    # 0.0968-0.0972 vs 0.0990-0.0997; B = 24: 0.1066-0.1080 vs 0.1111-0.1116,
    # profiles/r6aa_fused_gate_lines.txt; B = 64: 0.1948-0.1966 vs 0.1999-0.2042)
    if 2 * (x.shape[0] * heads) < _cu_count(x.device):
        return None
    return fz


_CUS: dict = {}


def _cu_count(dev: torch.device) -> int:
    n = _CUS.get(dev.index)
    if n is None:
        n = _CUS[dev.index] = torch.cuda.get_device_properties(dev).multi_processor_count
    return n


# large bf16 dense outputs also carry their fused per-tile sums (see hip._PSUM): y.sum() is free
_FUSED_SUM = os.environ.get("LJS_FUSED_SUM", "1") == "1"


# Deferred weight-gradient combines.  Inside value_and_grad on one device (no gradient
# all-reduce), a weight whose ONLY consumer is one _Linear (its AccumulateGrad node has a single
# incoming edge, from that _Linear's backward) gets its dW returned uncombined: the tensor autograd
# hands back is registered here with its split-K slabs, and value_and_grad wraps it in a LazyLocal
# whose ``slabs`` the fused Adam sums as it reads them (hip.SlabGrad) -- no slab_reduce launch.
# Anything else that reads the gradient forces the combine first.  Key: (data_ptr, shape).
_DEFER = None     # None, or {"safe": set of keys, "pending": {data_ptr: (descriptor, materialize)}}
_DEFER_ON = os.environ.get("LJS_DEFER_WGRAD", "1") == "1"


def _key(t: torch.Tensor):
    fn = t.grad_fn
    if fn is not None and type(fn).__name__ in _SLAB_CONSUMERS:
        # an output of a node that consumes its gradient as slabs (a gathered-weight proxy,
        # parallel/weight_gather.py): keyed by (node, output index)
        return ("node", id(fn), t.output_nr)
    return (t.data_ptr(), tuple(t.shape))


# autograd nodes that take their outputs' gradients uncombined (parallel/weight_gather.py: the
# loopback reduce-scatter of a gathered weight sums every device's split-K slabs in one pass)
_SLAB_CONSUMERS = ("_GatherBf16Backward",)


def defer_safe_leaves(outs, leaves: bool = True) -> set:
    """Keys of leaf tensors (``leaves``) and of slab-consumer outputs reached from ``outs`` by
    exactly one autograd edge, and that edge from a _Linear backward (so autograd passes that
    Function's gradient through untouched)."""
    counts, prod, seen = {}, {}, set()
    # (outs may hold autograd GradientEdges: a seed hoisted through an all-to-all, spmd.api)
    stack = [fn for fn in (t.grad_fn if isinstance(t, torch.Tensor) else t.node for t in outs) if fn is not None]
    while stack:
        fn = stack.pop()
        if id(fn) in seen:
            continue
        seen.add(id(fn))
        for nxt, idx in fn.next_functions:
            if nxt is None:
                continue
            var = getattr(nxt, "variable", None)
            k = None
            if var is not None:
                k = _key(var) if leaves else None
            elif type(nxt).__name__ in _SLAB_CONSUMERS:
                k = ("node", id(nxt), idx)
            if k is not None:
                counts[k] = counts.get(k, 0) + 1
                prod[k] = fn
            if var is None and id(nxt) not in seen:
                stack.append(nxt)
    return {k for k, c in counts.items() if c == 1 and type(prod[k]).__name__ in _DEFER_NODES}


# autograd nodes whose weight gradients may stay uncombined (they call _defer_ok per weight)
_DEFER_NODES = ("_LinearBackward", "_FFBlockBackward", "_FFBlockFp8Backward")


def defer_slabs(w: torch.Tensor, out: torch.Tensor, ld: int, offset: int = 0):
    """The ``defer`` callback of a weight-gradient GEMM writing ``out`` (= w's gradient, shape
    w.shape, element (r, c) at slab offset + r * ld + c), or None when w's gradient must be
    combined now (not inside a deferring value_and_grad, or w has another consumer)."""
    d = _DEFER
    if d is None or not _defer_ok(w) or tuple(out.shape) != tuple(w.shape) or out.dtype != torch.float32:
        return None
    pend = d["pending"]

    def defer(slabs, S, mat):
        pend[out.data_ptr()] = (hip.SlabGrad(slabs, S, offset, ld, slabs[0].numel(), tuple(out.shape)), mat)
    return defer


class defer_wgrads:
    """Context manager around one autograd.grad call (spmd.api.value_and_grad)."""

    def __init__(self, outs, enabled: bool, proxies: bool = False):
        """``enabled``: leaves' gradients may stay slabs (one device, the fused Adam sums them);
        ``proxies``: only slab-consumer outputs' may (several devices)."""
        self.state = None
        if (enabled or proxies) and _DEFER_ON:
            safe = defer_safe_leaves(outs, leaves=enabled)
            if safe:
                self.state = {"safe": safe, "pending": {}}

    def __enter__(self):
        global _DEFER
        self.prev, _DEFER = _DEFER, self.state
        return self

    def __exit__(self, *exc):
        global _DEFER
        flush_held_dw()
        _DEFER = self.prev
        return False

    def take(self, g: torch.Tensor):
        """(descriptor, materialize) if ``g`` is a returned gradient still uncombined, else None."""
        if self.state is None or g is None:
            return None
        ent = self.state["pending"].pop(g.data_ptr(), None)
        if ent is None:
            return None
        if tuple(ent[0].shape) != tuple(g.shape) or g.dtype != torch.float32 or not g.is_contiguous():
            ent[1]()
            return None
        return ent

    def flush(self):
        """Combine whatever was deferred but not handed back (nothing, when the safety walk holds)."""
        if self.state is not None:
            for _, mat in list(self.state["pending"].values()):
                mat()
            self.state["pending"].clear()


def _defer_ok(*ts) -> bool:
    d = _DEFER
    return d is not None and all(t is not None and t.dtype == torch.float32 and _key(t) in d["safe"] for t in ts)


# split-K weight-gradient slabs are f32 (bf16 slabs halved the slab bytes but measured no step gain
# and drifted the 2-rank 2-D parity past its tolerance: PERF_NOTES r4; removed in round 6)
_SLAB_DT = torch.float32


# Grouped weight-gradient launches (LJS_DW_GROUP=1, the default): inside a deferring backward
# (one device; the fused Adam reads the slabs after it) a slab-mode weight-gradient GEMM whose sums
# are deferred is held back as a job (its split count still open) and launched together with the
# NEXT one as one grid (hip.gemm_group_*: one block per work item of either, same kernel per item
# -> bit-identical), the pair's split counts chosen together (hip.pick_dw_pair: one round of
# resident blocks, equal-length items, fewer slabs).  At B = 64 the out-projection's and the QKV
# projection's dW GEMMs ran as 480 + 480 items (8 and 24 splits, 63 MB of slabs); paired they are
# 360 + 120 items of 6 splits each (31 MB).  Anything that reads a held GEMM's slabs launches it first.
_DW_GROUP = os.environ.get("LJS_DW_GROUP", "1") == "1"
# device index -> (held job, its stream); the lock: autograd runs one backward thread per device
_HELD: dict = {}
_HELD_LOCK = threading.RLock()


class _DwJob:
    """A held slab-mode weight-gradient GEMM: ``run(tile, S)`` allocates its S slabs, launches it
    and registers its deferred sums."""
    __slots__ = ("K", "N", "T", "tiles", "run")

    def __init__(self, K: int, N: int, T: int, tiles: int, run):
        self.K, self.N, self.T, self.tiles, self.run = K, N, T, tiles, run

    def run_alone(self):
        tile, S, _ = hip.pick_dw_slabs(self.K, self.N, self.T)
        self.run(tile, S)


def _group_ok(ref: torch.Tensor) -> bool:
    """Whether a slab-mode weight-gradient GEMM launched now may be grouped (see _DW_GROUP)."""
    return _DW_GROUP and _DEFER is not None and ref.is_cuda and not _DW_SPLIT


def deferred_pending():
    """The active deferral's pending map (gradient data_ptr -> (descriptor, materialize)), with any
    held weight-gradient GEMM launched first so its entries are in it; None outside a deferral."""
    if _DEFER is None:
        return None
    flush_held_dw()
    return _DEFER["pending"]


def flush_held_dw():
    """Launch the held weight-gradient GEMMs (if any) on their own, each on its own stream."""
    if not _HELD:
        return
    with _HELD_LOCK:
        while _HELD:
            _, (job, st) = _HELD.popitem()
            if st is None:
                job.run_alone()
                continue
            with torch.cuda.stream(st):
                job.run_alone()


def _hold_dw(job: _DwJob, ref: torch.Tensor) -> None:
    """Hold ``job`` to be grouped with the next one on its device, or launch it with the held one
    as a pair."""
    stream = torch.cuda.current_stream(ref.device) if ref.is_cuda else None
    with _HELD_LOCK:
        held = _HELD.pop(ref.device.index, None)
        if held is None:
            _HELD[ref.device.index] = (job, stream)
            return
        prev, pst = held
        if pst != stream:
            with torch.cuda.stream(pst):
                prev.run_alone()
            _HELD[ref.device.index] = (job, stream)
            return
        pick = hip.pick_dw_pair(prev.K, prev.N, job.K, job.N, job.T) if prev.T == job.T else None
        if pick is None:
            prev.run_alone()
            job.run_alone()
            return
        tile, s0, s1 = pick
        hip.gemm_group_begin()
        try:
            prev.run(tile, s0)
            job.run(tile, s1)
        finally:
            hip.gemm_group_end(ref)


def _dw_slabs_wmajor(xb: torch.Tensor, dys, T: int, K: int, N: int, ws, pend):
    """The weight gradients xb^T @ dys[i] of weight-major cotangents dys [nw][T][N] (a seq-major
    fused projection, ops.linear.token_outer) as ONE slab-mode launch (batch i, split s -> slab
    [s][i] of [S][nw][K][N]) and, when combined, ONE slab_reduce into views of one [nw][K][N]
    buffer (so a reduce-scatter / bucket takes them without a concatenation).  Each gradient is
    deferred as slabs when allowed (``pend``).  None when the slab-mode kernel does not apply."""
    nw = len(ws)
    tile, S, slab_mode = hip.pick_dw_slabs(K, nw * N, T)
    if not slab_mode or (_DW_SPLIT and T % (64 * _DW_SPLIT) == 0):
        return None
    out = torch.empty((nw, K, N), dtype=torch.float32, device=xb.device)
    deferred = [pend is not None and _defer_ok(w) for w in ws]

    def run(tile, S):
        slabs = torch.empty((S, nw, K, N), dtype=_SLAB_DT, device=xb.device)
        # dys: the nw [T][N] cotangents (separate tensors: q's from the attention backward, k's and
        # v's from the sequence gather's reduce-scatter), read through per-batch B pointers
        hip.gemm(xb, dys[0], slabs, K, N, T, K, N, N, False, False, batch=nw, sA=0, sC=K * N, splitk=S,
                 tile=tile, slabs=True, b_list=dys)
        done = []

        def materialize():
            if not done:
                done.append(True)
                flush_held_dw()
                hip.slab_reduce(slabs.view(S, nw * K, N), out.view(nw * K, N), N, 0)
        for i in range(nw):
            if deferred[i]:
                pend[out[i].data_ptr()] = (hip.SlabGrad(slabs, S, i * K * N, N, nw * K * N, (K, N)), materialize)
            else:
                materialize()
    if all(deferred) and _group_ok(xb):
        _hold_dw(_DwJob(K, nw * N, T, nw * -(-K // 128) * -(-N // 128), run), xb)
    else:
        run(tile, S)
    return [out[i] for i in range(nw)]


def _dw_slabs(xb: torch.Tensor, dy: torch.Tensor, ld: int, T: int, K: int, Nt: int, out: torch.Tensor, cb: int,
              out_bs: int, twin: Optional[torch.Tensor] = None, tail=None, defer=None) -> None:
    """out (column blocks of width cb, out_bs apart) = xb^T @ dy for xb [T][K], dy [T][Nt] (row
    stride ld, 0 = broadcast row): S K-chunks of the token dim run as one batched LDS-DMA GEMM
    into f32 slabs [S][K][Nt], combined by one streaming reduction (which also fills ``tail`` =
    (f32 tensor, bf16 twin or None, constant)).  ``defer(slabs, S, materialize)``: the
    reduction is not launched; ``materialize()`` runs it (once) if the sums are ever read."""
    tile, S, slab_mode = hip.pick_dw_slabs(K, Nt, T)
    if _DW_SPLIT and T % (64 * _DW_SPLIT) == 0:
        S, slab_mode = _DW_SPLIT, False

    def run(tile, S):
        slabs = torch.empty((S, K, Nt), dtype=_SLAB_DT if slab_mode else torch.float32, device=xb.device)
        if slab_mode:  # one launch, split s of the token range into slab s (uneven last split)
            hip.gemm(xb, dy, slabs, K, Nt, T, K, ld, Nt, False, False, sC=K * Nt, splitk=S, tile=tile, slabs=True)
        else:
            kc = T // S
            hip.gemm(xb, dy, slabs, K, Nt, kc, K, ld, Nt, False, False, batch=S, sA=kc * K, sB=kc * ld,
                     sC=K * Nt, tile=tile)
        done = []

        def materialize():
            if done:
                return
            done.append(True)
            flush_held_dw()
            if tail is not None:
                hip.slab_reduce(slabs, out, cb, out_bs, out_bf16=twin, tail=tail[0], tail_bf16=tail[1],
                                tail_val=tail[2])
            else:
                hip.slab_reduce(slabs, out, cb, out_bs, out_bf16=twin)
        if defer is not None:
            defer(slabs, S, materialize)
        else:
            materialize()
    if slab_mode and defer is not None and _group_ok(xb):
        _hold_dw(_DwJob(K, Nt, T, -(-K // 128) * -(-Nt // 128), run), xb)
    else:
        run(tile, S)


def _row_view(dy: torch.Tensor, M: int, N: int) -> Tuple[torch.Tensor, int]:
    """(bf16 tensor, ld) describing dy as an [M][N] matrix with unit column stride.

    A gradient that repeats one row (stride 0 over rows, e.g. the cotangent of ``y.sum()``)
    is returned as that single bf16 row with ld = 0: the GEMMs and the column sum read it
    M times, exactly as they would read a materialised matrix, without writing one.
    """
    d2 = dy.reshape(M, N)
    if d2.is_cuda and d2.numel() > 0 and d2.stride(0) == 0 and d2.stride(1) == 0:
        # one broadcast scalar (the cotangent of y.sum()): a cached constant row when it is a
        # constant seed, else its bf16 row in one HIP launch (a torch .contiguous() of the
        # stride-0 row ran as a 1-workgroup copy kernel, ~4.7 us)
        g1 = d2.as_strided((1,), (1,))
        cval = hip.seed_constant(g1)
        row = hip.const_row_bf16(cval, N, d2.device) if cval is not None else None
        if row is None:
            row, _ = hip.bcast_scalar(g1, N, M, False)
        return row.unsqueeze(0).expand(M, N), 0
    if d2.stride(0) == 0:
        row = d2[0].contiguous()
        row = _bf16(row)
        return row.unsqueeze(0).expand(M, N), 0
    if d2.stride(1) != 1 or d2.stride(0) < N:
        d2 = d2.contiguous()
    if d2.dtype != torch.bfloat16:
        d2 = _bf16(d2.contiguous())
    return d2, d2.stride(0)


# ops.core.dense's layout hint: the logical dim to keep OUTERMOST in the outputs' storage
# (1 = the sequence of a (batch, seq, features) activation whose sequence is sharded)
_TOKEN_OUTER: List[Optional[int]] = [None]


class token_outer:
    """Context: dense layers called inside produce ``dim``-major outputs (see _row_order)."""

    def __init__(self, dim: Optional[int]):
        self.dim = dim

    def __enter__(self):
        self.prev, _TOKEN_OUTER[0] = _TOKEN_OUTER[0], self.dim
        return self

    def __exit__(self, *exc):
        _TOKEN_OUTER[0] = self.prev
        return False


def _inv_perm(order):
    inv = [0] * len(order)
    for i, d in enumerate(order):
        inv[d] = i
    return tuple(inv)


def _row_order(x: torch.Tensor):
    """(dim order with the feature dim last, swap): the order in which x's leading dims are
    flattened into GEMM rows - x's own storage order when x is dense with its feature dim
    innermost, else logical order.  ``swap``: x is a contiguous (batch, seq, K) activation and the
    active hint asks for seq-major rows - it is transposed while being rounded to bf16."""
    nd = x.dim()
    ident = tuple(range(nd))
    o = hip.storage_order(x) if x.is_cuda else None
    if o is not None and o[-1] == nd - 1 and o != ident:
        return tuple(o), False
    hint = _TOKEN_OUTER[0]
    if (hint == 1 and nd == 3 and x.is_cuda and x.is_contiguous() and x.shape[0] > 1 and x.shape[1] > 1
            and x.shape[2] % 8 == 0 and x.dtype in (torch.float32, torch.bfloat16) and x.data_ptr() % 16 == 0):
        return (1, 0, 2), True
    return ident, False


def _bf16(t: torch.Tensor) -> torch.Tensor:
    if t.dtype == torch.bfloat16:
        return t
    if t.is_contiguous():
        pre = _take_precast(t)
        if pre is not None:
            return pre
        return hip._cast_raw(t, torch.bfloat16)
    return t.to(torch.bfloat16)


# ---------------------------------------------------------------------------- input-cast prefetch
# The reference's f32 activation is rounded to bf16 inside its first Dense (case6_attention.py:
# 96-99); here that is a streaming cast pass in front of the QKV GEMM (11 us at 64 x 256 tokens).
# A multi-step runner that knows the NEXT step's input registers it (`prefetch_next_input`) before
# running a step; the cast of that input is then queued earlier, where it costs less, and the next
# step's dense takes the copy (`_take_precast`) instead of casting.  Every step still casts its
# own input exactly once: only WHEN changes.  Runners drop what was not taken (`join_precasts`)
# before their capture ends.
#  * single-process steps: the optimizer launch's extra blocks cast it (hip.adam_multi,
#    `take_optimizer_precast`): B = 8 0.0719-0.0729 vs 0.0736-0.0742 ms (profiles/
#    r5bb_opt_precast_lines.txt);
#  * data-parallel steps: queued on the step's own stream just before the backward waits for its
#    gradient all-reduce (parallel/data.GradReducer.finish, `launch_join_precasts`), where the
#    stream would otherwise idle behind the collective's tail.
# Only inputs whose cast the forward runs as the plain pass (not a transposing or fused path) are
# cast early.  (A side-stream form -- the cast forked beside the backward -- measured much slower:
# B=64 0.2472 vs 0.2180 ms, profiles/r5t_precast_lines.txt; removed.)  LJS_PRECAST=0: off.
_PRECAST_MODE = os.environ.get("LJS_PRECAST", "join")
_NEXT_INPUTS: List[torch.Tensor] = []
_PLAIN_CAST = set()      # (numel, device index) of next-step inputs the forward cast plainly
PRECAST_STATS = {"taken": 0}
_PRECAST = {}            # key -> (bf16 copy, source)
# LJS_OPT_PRECAST=0: single-process steps keep the next input's cast in its own forward
_OPT_PRECAST = os.environ.get("LJS_OPT_PRECAST", "1")


def _pc_key(t: torch.Tensor):
    return (t.data_ptr(), t.numel(), t._version, t.device.index)


def prefetch_next_input(*xs) -> None:
    """Register the next step's input(s) (tensors or sharded arrays; f32 CUDA shards only) for
    an early bf16 cast during the coming step."""
    if _PRECAST_MODE == "0":
        return
    _register_capture_hook()
    for x in xs:
        loc = getattr(x, "local", None)
        ts = list(loc.values()) if isinstance(loc, dict) else [x]
        for t in ts:
            if (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
                    and t.numel() >= (1 << 20)):
                _NEXT_INPUTS.append(t)


def _single_device_capture() -> bool:
    from ..spmd import graphs as _graphs
    return not isinstance(_graphs.current(), _graphs.MultiDeviceGraph)


def launch_join_precasts() -> None:
    """Cast the registered next-step inputs now, on the current stream (called before a
    data-parallel backward joins its gradient all-reduce)."""
    if _PRECAST_MODE == "0" or not _NEXT_INPUTS:
        return
    if not _single_device_capture():
        _NEXT_INPUTS.clear()
        return
    todo = [t for t in _NEXT_INPUTS if (t.numel(), t.device.index) in _PLAIN_CAST]
    _NEXT_INPUTS.clear()
    for t in todo:
        k = _pc_key(t)
        if k not in _PRECAST:
            _PRECAST[k] = (hip._cast_raw(t.reshape(-1), torch.bfloat16), t)


def take_optimizer_precast(dev: torch.device):
    """(f32 source, bf16 destination, input) of ONE registered next-step input on ``dev`` that the
    optimizer launch casts with its extra blocks (hip.adam_multi) -- or None.  The destination
    becomes that input's early cast only once the launch that writes it has been accepted
    (:func:`commit_optimizer_precast`): a rejected launch leaves no unwritten buffer registered."""
    if _PRECAST_MODE == "0" or not _NEXT_INPUTS or _OPT_PRECAST == "0" or not _single_device_capture():
        return None
    for i, t in enumerate(_NEXT_INPUTS):
        if (t.device == dev and (t.numel(), t.device.index) in _PLAIN_CAST and t.is_contiguous()
                and t.data_ptr() % 16 == 0 and _pc_key(t) not in _PRECAST):
            del _NEXT_INPUTS[i]
            dst = torch.empty(t.shape, dtype=torch.bfloat16, device=t.device)
            return t.reshape(-1), dst.reshape(-1), t
    return None


def commit_optimizer_precast(cast) -> None:
    """Register the early cast of :func:`take_optimizer_precast` after its launch succeeded."""
    src, dst, t = cast
    _PRECAST[_pc_key(t)] = (dst.view(t.shape), t)


def _take_precast(t: torch.Tensor):
    if _NEXT_INPUTS and t.is_cuda and t.dtype == torch.float32 and any(
            n.numel() == t.numel() and n.device == t.device for n in _NEXT_INPUTS):
        # a registered next-step input cast by the plain pass (a [tokens, features] view of
        # it): worth casting early
        _PLAIN_CAST.add((t.numel(), t.device.index))
    if not _PRECAST or not t.is_cuda:
        return None
    ent = _PRECAST.pop(_pc_key(t), None)
    if ent is None:
        return None
    PRECAST_STATS["taken"] += 1
    return ent[0].view(t.shape)


def join_precasts() -> None:
    """Forget every early cast nobody took and drop pending registrations -- call before a
    capture or a step sequence ends (a whole capture's end does it too)."""
    _NEXT_INPUTS.clear()
    _PRECAST.clear()


def _register_capture_hook() -> None:
    from ..spmd import graphs as _graphs
    if join_precasts not in _graphs.AFTER_CAPTURE:
        _graphs.AFTER_CAPTURE.append(join_precasts)


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b, res, relu, out_dtype, *ws):
        lead = x.shape[:-1]
        K = x.shape[-1]
        # rows (tokens) in x's STORAGE order: a seq-major activation ((batch, seq, K) stored
        # [seq][batch][K]) is flattened without a copy and the outputs keep that order
        order, swap = _row_order(x)
        x2 = x.permute(order).reshape(-1, K) if not swap else None
        M = x.numel() // max(1, K)
        nw = len(ws)
        N = ws[0].shape[1]
        pshape = tuple(x.shape[d] for d in order[:-1])
        inv = _inv_perm(order)
        # weight-major outputs ([nw][M][N]: each projection dense on its own) for a seq-major
        # fused projection, so its K / V gather over the sequence are contiguous blocks
        wmajor = nw > 1 and order[0] != 0
        # f32 activations (the reference's f32 input under a bf16 Dense) are rounded by one cast
        # pass -- or, for a multi-step runner's next input, by the previous step's optimizer launch
        # (take_optimizer_precast).  Rounding inside the GEMM (an f32 A operand, LDS image or
        # register-staged) measured slower in both forms and was removed (PERF_NOTES r2, r4).
        if swap:   # batch-major x -> seq-major bf16 rows, rounded in the same pass
            xb = hip.swap01_bf16(x.contiguous()).view(M, K)
        else:
            xb = _bf16(x2 if x2.is_contiguous() else x2.contiguous())
        # weights gathered on a side stream (parallel/fsdp.Prefetcher.prefetch(defer_wait=True)):
        # the stream waits for them only now, after the activation's cast pass was queued
        take_pending_waits(x.device)
        if nw == 1:
            wt = shadow.get(ws[0], "T")
            sB = 0
        else:
            # one [nw][N][K] operand: the weights' transposed shadows live in one allocation
            wt = shadow.get_stacked(ws)
            sB = N * K
        od = out_dtype if out_dtype in (torch.bfloat16, torch.float32) else torch.float32
        out = torch.empty((nw, M, N) if wmajor else (M, nw * N), dtype=od, device=x.device)
        bias = None
        if b is not None:
            bias = (b if b.dtype in (torch.float32, torch.bfloat16) else b.float()).contiguous()
        partials = None
        if _FUSED_SUM and nw == 1 and od == torch.bfloat16 and M * N >= (1 << 20):
            partials = torch.empty((hip.psum_slots(M, N),), dtype=torch.float32, device=x.device)
        # residual fused into the epilogue (bf16 output, one kernel, 8-column-aligned operand)
        r2, r_ld = None, 0
        if res is not None:
            if (order == (1, 0, 2) and res.dim() == 3 and res.is_cuda and res.is_contiguous() and N % 8 == 0
                    and res.dtype in (torch.float32, torch.bfloat16) and res.data_ptr() % 16 == 0
                    and res.shape[1] <= 65535):
                # a batch-major residual under seq-major rows (the 2-D mesh's out projection with the
                # layer's skip x): one transposing pass that also rounds to bf16 - the epilogue rounds
                # the residual to bf16 before the add anyway - instead of an f32 transposing copy
                r2 = hip.swap01_bf16(res).view(M, N)
            else:
                r2 = res.permute(order).reshape(M, N)
            if r2.dtype not in (torch.bfloat16, torch.float32):
                r2 = r2.float()
            if not (r2.stride(1) == 1 and r2.stride(0) % 8 == 0 and r2.data_ptr() % 16 == 0):
                r2 = r2.contiguous()
            r_ld = r2.stride(0)
            if nw != 1 or od != torch.bfloat16 or N % 8:
                r2 = None
        fz = _fuse_attention_ok(x, xb, wt, nw, N, K, b, relu, res, od, out_dtype, wmajor, order, swap)
        if fz is not None:
            o_att, lse_att = hip.qkv_attn_fwd(xb, wt, out, fz[0], fz[2])
            hip.register_fused_attention(out, o_att, lse_att, fz[0], fz[2])
            cnt = 0
        else:
            cnt = hip.gemm(xb, wt, out, M, N, K, K, K, N if wmajor else nw * N, True, True, batch=nw, sA=0, sB=sB,
                           sC=M * N if wmajor else N, bias=bias, sBias=0, relu=relu, psum=partials, res=r2,
                           res_ld=r_ld)
        cols = [out[i] if wmajor else out[:, i * N:(i + 1) * N] for i in range(nw)]
        ys = [c.view(pshape + (N,)).permute(inv) for c in cols]
        if res is not None and r2 is None:
            ys = [ys[0] + res.to(ys[0].dtype)]
            partials = None
        if partials is not None and cnt > 0 and od == out_dtype:
            hip._register_psum(ys[0], partials, cnt)
        if od != out_dtype:
            ys = [y.to(out_dtype) for y in ys]
        if relu and od == torch.bfloat16:
            for y in ys:
                _register(_RELU_OUT, y)
        # this dense's input is a ReLU output: its dX GEMM can apply that ReLU's backward mask.
        # Keyed on autograd identity as well as storage: x must come straight out of a ReLU
        # dense's backward node (a .detach()ed copy shares the storage but not the graph edge)
        ctx.premask = bool(xb.dtype == torch.bfloat16 and K % 8 == 0 and _is_relu_out(xb) and _relu_node(x))
        ctx.has_res = res is not None
        ctx.save_for_backward(xb, b, *ws, *(ys if relu else []))
        ctx.meta = (lead, K, M, N, nw, relu, x.dtype, b is not None)
        ctx.order, ctx.pshape = order, pshape
        return tuple(ys)

    @staticmethod
    def backward(ctx, *dys):
        lead, K, M, N, nw, relu, xdtype, has_b = ctx.meta
        order = getattr(ctx, "order", None)          # (the fp8 dense reuses this backward in row order)
        pshape = ctx.pshape if order is not None else tuple(lead)
        if order is None:
            order = tuple(range(len(lead) + 1))
        # the residual's gradient is the output gradient itself (y = dense(x) + res)
        dres = dys[0] if (ctx.has_res and ctx.needs_input_grad[2]) else None
        # every [M][N] view below is in the forward's row (storage) order
        dys = tuple(None if d is None else d.permute(order) for d in dys)
        saved = ctx.saved_tensors
        xb, b = saved[0], saved[1]
        ctx.bias_leaf = b
        ws = saved[2:2 + nw]
        ys = tuple(y.permute(order) for y in saved[2 + nw:]) if relu else None
        dev = xb.device
        mats: List[Optional[Tuple[torch.Tensor, int]]] = []
        db_bcast: List[Optional[torch.Tensor]] = [None] * nw
        want_db = has_b and ctx.needs_input_grad[1]
        # one dense with a bias whose cotangent is a scalar broadcast (a loss sum), both gradients
        # wanted: dW and db share ONE f32 buffer [K*N + N]
        # (and, under a bf16 data-parallel wire, one bf16 twin) so the gradient all-reduce sends
        # them as one producer group -- no concatenation, no cast kernel (parallel/data.py)
        from ..parallel import data as _dp
        wire = _dp.active_wire_dtype() == torch.bfloat16
        joint = joint_bf16 = tail = None
        if (nw == 1 and want_db and ctx.needs_input_grad[5] and dys[0] is not None and M % 64 == 0 and not relu
                and b.dtype == torch.float32 and ws[0].dtype == torch.float32 and dys[0].is_cuda
                and dys[0].numel() > 0 and all(st == 0 for st in dys[0].stride())):
            joint = torch.empty((K * N + N,), dtype=torch.float32, device=dev)
            joint_bf16 = torch.empty((K * N + N,), dtype=torch.bfloat16, device=dev) if wire else None
        for i, dy in enumerate(dys):
            if dy is None:
                mats.append(None)
                continue
            if relu and _premasked_by(dy, ys[i]):
                # the consumer's dX GEMM already applied this ReLU's mask
                mats.append(_row_view(dy, M, N))
                continue
            if relu:
                d2, y2 = dy.reshape(M, N), ys[i].reshape(M, N)
                if (d2.is_cuda and d2.dtype == torch.bfloat16 and y2.dtype == torch.bfloat16 and N % 8 == 0
                        and d2.stride(1) == 1 and y2.stride(1) == 1 and d2.stride(0) % 8 == 0
                        and y2.stride(0) % 8 == 0 and d2.data_ptr() % 16 == 0 and y2.data_ptr() % 16 == 0):
                    # fused ReLU backward: the masked gradient and its column sums (the bias
                    # gradient) in one pass over dy and y
                    if want_db:
                        masked, db_bcast[i] = hip.relu_bwd_colsum(d2, y2, M, N)
                    else:  # no bias gradient wanted: a flat full-chip pass, no column sums
                        masked = hip.relu_bwd(d2, y2, M, N)
                    mats.append((masked, N))
                    continue
                dy = (dy * (ys[i] > 0)).reshape(M, N)
            elif dy.is_cuda and dy.numel() > 0 and all(st == 0 for st in dy.stride()):
                # one scalar broadcast (the cotangent of y.sum()): its bf16 row and the bias
                # gradient come out of one kernel; the GEMMs read the row with ld = 0.  A constant
                # seed's row is a cached constant and its bias gradient M * bf16(g) is written by
                # the weight-gradient combine into the joint buffer: no launch at all
                g1 = dy.as_strided((1,), (1,))
                cval = hip.seed_constant(g1) if joint is not None else None
                row = hip.const_row_bf16(cval, N, dev) if cval is not None else None
                if row is not None:
                    db_bcast[i] = joint[K * N:]
                    tail = (joint[K * N:], joint_bf16[K * N:] if joint_bf16 is not None else None,
                            float(np.float32(cval) * np.float32(M)))
                    mats.append((row.unsqueeze(0).expand(M, N), 0))
                    continue
                row, db_bcast[i] = hip.bcast_scalar(
                    dy.as_strided((1,), (1,)), N, M, want_db,
                    db_out=joint[K * N:] if joint is not None else None,
                    db_bf16=joint_bf16[K * N:] if joint_bf16 is not None else None)
                mats.append((row.unsqueeze(0).expand(M, N), 0))
                continue
            mats.append(_row_view(dy, M, N))
        dx = db = None
        dws = [None] * nw
        live = [i for i in range(nw) if mats[i] is not None]
        # ---- dX
        if ctx.needs_input_grad[0] and live:
            out_dt = torch.bfloat16 if (xdtype == torch.bfloat16 and len(live) == 1) else torch.float32
            dx = torch.empty((M, K), dtype=out_dt, device=dev)
            premask = ctx.premask and out_dt == torch.bfloat16
            for j, i in enumerate(live):
                t, ld = mats[i]
                wn = shadow.get(ws[i], "N")                  # [K][N]: B[k=n][n'=k], k-contiguous
                hip.gemm(t, wn, dx, M, K, N, ld, N, K, True, True, accumulate=j > 0,
                         res=xb if premask else None, res_ld=K, res_mode="mask")
            dx = dx.to(xdtype).view(pshape + (K,)).permute(_inv_perm(order))
            if premask:
                _register(_PREMASKED, dx, xb.data_ptr())
        # ---- dW (MN-contiguous operands: X^T and dY read in place), on the compute stream (a side
        # stream overlapping the input-gradient chain measured slower at every bench shape: two
        # chip-sized persistent grids share the CUs as two rounds + a tail, PERF_NOTES r2; removed)
        want = [i for i in live if ctx.needs_input_grad[5 + i]]
        _wgrads(ctx, xb, ws, mats, want, dws, joint, joint_bf16, K, M, N, nw, wire, dev, tail)
        # ---- db
        if want_db and live:
            tot = None
            for i in live:
                if db_bcast[i] is not None:
                    tot = db_bcast[i] if tot is None else tot + db_bcast[i]
                    continue
                t, ld = mats[i]
                pre = hip.colsum_for(t, N) if ld > 0 else None
                if pre is not None:   # the loss kernel that produced dY summed its columns already
                    tot = pre if tot is None else tot + pre
                    continue
                tot = hip.colsum_ld(t, M, N, ld, tot)
            db = tot.to(b.dtype)
        if joint is not None:
            if dws[0] is None or db is None or db.data_ptr() != joint[K * N:].data_ptr():
                joint_bf16 = None  # the two gradients did not both land in the joint buffer
            if joint_bf16 is not None:
                _dp.register_wire_twin(joint, joint_bf16)
        return (dx, db, dres, None, None, *dws)


# side-stream gathers whose completion the next _Linear forward waits for after its input cast
_PENDING_WAITS: List = []


def defer_wait(handle) -> None:
    """Register a prefetch handle (parallel/fsdp._Handle) to be waited on by the next dense GEMM
    after it has queued its activation pass; the caller still calls ``handle.wait()`` after the
    dense (a no-op for the stream by then) in case no GEMM consumed it."""
    _PENDING_WAITS.append(handle)


def take_pending_waits(dev) -> None:
    while _PENDING_WAITS:
        _PENDING_WAITS.pop().wait()


def twin_free(joint_bf16, wire) -> bool:
    return joint_bf16 is None and not wire


def _wgrads(ctx, xb, ws, mats, want, dws, joint, joint_bf16, K, M, N, nw, wire, dev, tail=None):
    """The weight gradients of :class:`_Linear` (``dws[i]`` for ``i`` in ``want``)."""
    from ..parallel import data as _dp
    if not want:
        return
    t0, ld0 = mats[want[0]]
    batched = (len(want) == nw and nw > 1 and ld0 > 0 and all(
        mats[i][1] == ld0 and mats[i][0].data_ptr() == t0.data_ptr() + i * N * 2 for i in want))
    dma = M % 64 == 0
    if dma:
        # split-K as a batch over K-chunks writing per-chunk f32 slabs, then one combine
        # pass (no atomics, no memset): the column blocks of a fused [K][nw*N] product are
        # the nw weight gradients
        # under a data-parallel backward with a bf16 gradient wire, the combine also writes
        # the bf16 twin the all-reduce sends (no separate cast kernel; parallel/data.py)
        pend = _DEFER["pending"] if _DEFER is not None and twin_free(joint_bf16, wire) else None
        if joint is not None:
            t, ld = mats[0]
            dW = joint[:K * N].view(K, N)
            defer = None
            if pend is not None and _defer_ok(ws[0], *([ctx.bias_leaf] if tail is not None else [])):
                def defer(slabs, S, mat, dW=dW):
                    pend[dW.data_ptr()] = (hip.SlabGrad(slabs, S, 0, N, K * N, (K, N)), mat)
                    if tail is not None:
                        pend[tail[0].data_ptr()] = (hip.ConstGrad(tail[2], (N,)), mat)
            _dw_slabs(xb, t, ld, M, K, N, dW, N, 0,
                      joint_bf16[:K * N].view(K, N) if joint_bf16 is not None else None, tail, defer)
            dws[0] = dW
        elif batched:
            dW = torch.empty((nw, K, N), dtype=torch.float32, device=dev)
            twin = torch.empty((nw, K, N), dtype=torch.bfloat16, device=dev) if wire else None
            defer = None
            if pend is not None and twin is None and _defer_ok(*[ws[i] for i in want]):
                def defer(slabs, S, mat, dW=dW):
                    for i in want:
                        pend[dW[i].data_ptr()] = (hip.SlabGrad(slabs, S, i * N, nw * N, K * nw * N, (K, N)), mat)
            _dw_slabs(xb, t0, ld0, M, K, nw * N, dW, N, K * N, twin, defer=defer)
            if twin is not None:
                _dp.register_wire_twin(dW, twin)
            for i in want:
                dws[i] = dW[i] if ws[i].dtype == torch.float32 else dW[i].to(ws[i].dtype)
        elif (_WMAJOR_BATCH and len(want) == nw and 1 < nw <= 4 and not wire and all(
                mats[i][1] == N and mats[i][0].stride(-1) == 1 and mats[i][0].data_ptr() % 16 == 0 for i in want)
                and (wm := _dw_slabs_wmajor(xb, [mats[i][0] for i in want], M, K, N, [ws[i] for i in want],
                                            pend)) is not None):
            for j, i in enumerate(want):
                dws[i] = wm[j] if ws[i].dtype == torch.float32 else wm[j].to(ws[i].dtype)
        else:
            for i in want:
                t, ld = mats[i]
                dW = torch.empty((K, N), dtype=torch.float32, device=dev)
                twin = torch.empty((K, N), dtype=torch.bfloat16, device=dev) if wire else None
                defer = None
                if pend is not None and twin is None and _defer_ok(ws[i]):
                    def defer(slabs, S, mat, dW=dW):
                        pend[dW.data_ptr()] = (hip.SlabGrad(slabs, S, 0, N, K * N, (K, N)), mat)
                _dw_slabs(xb, t, ld, M, K, N, dW, N, 0, twin, defer=defer)
                if twin is not None:
                    _dp.register_wire_twin(dW, twin)
                dws[i] = dW if ws[i].dtype == torch.float32 else dW.to(ws[i].dtype)
    else:
        tile = 128 if (K >= 256 and N >= 256) else 64
        if batched:
            dW = torch.empty((nw, K, N), dtype=torch.float32, device=dev)
            sk = _splitk(K, N, M, nw, tile)
            hip.gemm(xb, t0, dW, K, N, M, K, ld0, N, False, False, batch=nw, sA=0, sB=N, sC=K * N,
                     splitk=sk, tile=tile, zero_c=True)
            for i in want:
                dws[i] = dW[i] if ws[i].dtype == torch.float32 else dW[i].to(ws[i].dtype)
        else:
            for i in want:
                t, ld = mats[i]
                dW = torch.empty((K, N), dtype=torch.float32, device=dev)
                sk = _splitk(K, N, M, 1, tile)
                hip.gemm(xb, t, dW, K, N, M, K, ld, N, False, False, splitk=sk, tile=tile, zero_c=True)
                dws[i] = dW if ws[i].dtype == torch.float32 else dW.to(ws[i].dtype)


# the weight-major (seq-major fused projection) weight gradients as one batched slab-mode launch
# instead of one GEMM per weight (LJS_WMAJOR_DW_BATCH=0: per weight)
_WMAJOR_BATCH = os.environ.get("LJS_WMAJOR_DW_BATCH", "1") == "1"


def supported(x: torch.Tensor, ws: Sequence[torch.Tensor], b) -> bool:
    K = x.shape[-1]
    N = ws[0].shape[1]
    M = x.numel() // max(1, K)   # the weight-gradient GEMM contracts over the M rows
    return (K % 8 == 0 and N % 8 == 0 and M % 8 == 0 and all(w.shape == ws[0].shape and w.dim() == 2 for w in ws)
            and all(w.dtype == torch.float32 and w.stride(1) == 1 for w in ws)
            and (b is None or len(ws) == 1))


def linear(x: torch.Tensor, ws: List[torch.Tensor], b: Optional[torch.Tensor], relu: bool,
           out_dtype: torch.dtype, residual: Optional[torch.Tensor] = None) -> List[torch.Tensor]:
    if residual is not None and (relu or len(ws) != 1):
        # the epilogue adds the residual after the activation; a ReLU dense keeps its own output
        # for the backward mask, so that combination adds separately
        ys = list(_Linear.apply(x, b, None, relu, out_dtype, *ws))
        return [ys[0] + residual.to(ys[0].dtype)] + ys[1:]
    return list(_Linear.apply(x, b, residual, relu, out_dtype, *ws))


# ----------------------------------------------------------------------------- fused FF block
class _FFBlock(torch.autograd.Function):
    """``y = relu(x Win) Wout + x`` (the transformer layer's FF sub-block with its skip
    connection; ``res`` False: without it) as ONE autograd node, so the gradient of x - the
    skip path's dY plus the FF path's dX - is summed inside the dX GEMM's epilogue instead of
    by a separate autograd accumulation kernel:

    * forward: up projection with ReLU, down projection with the residual in its epilogue;
    * backward: dA = dY Wout^T with the ReLU mask in the epilogue; dX = dA Win^T (+ dY, the
      residual, in the epilogue, bit-exact with the separate bf16 add); weight gradients as
      split-K slabs (+ bf16 wire twins under a bf16 data-parallel wire)."""

    @staticmethod
    def forward(ctx, x, w_in, w_out, res):
        M = x.shape[-1]
        F = w_in.shape[1]
        # tokens in x's storage order (a seq-major activation is read without a transposing copy;
        # y and dX keep its layout), as in _Linear
        nd = x.dim()
        o = hip.storage_order(x) if x.is_cuda else None
        order = tuple(o) if o is not None and o[-1] == nd - 1 else tuple(range(nd))
        xs = x.permute(order)
        pshape = tuple(xs.shape[:-1])
        x2 = _bf16(xs.reshape(-1, M).contiguous())
        T = x2.shape[0]
        a = torch.empty((T, F), dtype=torch.bfloat16, device=x.device)
        hip.gemm(x2, shadow.get(w_in, "T"), a, T, F, M, M, M, F, True, True, relu=True)
        y = torch.empty((T, M), dtype=torch.bfloat16, device=x.device)
        hip.gemm(a, shadow.get(w_out, "T"), y, T, M, F, F, F, M, True, True, res=x2 if res else None, res_ld=M)
        ctx.save_for_backward(x2, a, w_in, w_out)
        ctx.meta = (order, pshape, M, F, T, bool(res), x.dtype)
        return y.view(pshape + (M,)).permute(_inv_perm(order))

    @staticmethod
    def backward(ctx, dy):
        from ..parallel import data as _dp
        x2, a, w_in, w_out = ctx.saved_tensors
        order, pshape, M, F, T, res, xdt = ctx.meta
        dev = x2.device
        t, ld = _row_view(dy.permute(order), T, M)
        wire = _dp.active_wire_dtype() == torch.bfloat16
        dA = torch.empty((T, F), dtype=torch.bfloat16, device=dev)
        hip.gemm(t, shadow.get(w_out, "N"), dA, T, F, M, ld, M, F, True, True, res=a, res_ld=F, res_mode="mask")
        out = {}

        def run_dx():
            if ctx.needs_input_grad[0]:
                dx = torch.empty((T, M), dtype=torch.bfloat16, device=dev)
                hip.gemm(dA, shadow.get(w_in, "N"), dx, T, M, F, F, F, M, True, True, res=t if res else None,
                         res_ld=ld)
                out["dx"] = dx.to(xdt).view(pshape + (M,)).permute(_inv_perm(order))

        def wgrad(xb, g, g_ld, K, N, w):
            o = torch.empty((K, N), dtype=torch.float32, device=dev)
            twin = torch.empty((K, N), dtype=torch.bfloat16, device=dev) if wire else None
            _dw_slabs(xb, g, g_ld, T, K, N, o, N, 0, twin, defer=defer_slabs(w, o, N) if twin is None else None)
            if twin is not None:
                _dp.register_wire_twin(o, twin)
            return o

        def run_wo():
            if ctx.needs_input_grad[2]:
                out["wo"] = wgrad(a, t, ld, F, M, w_out)

        def run_wi():
            if ctx.needs_input_grad[1]:
                out["wi"] = wgrad(x2, dA, F, M, F, w_in)
        _ff_bwd_order(run_dx, run_wo, run_wi)
        return out.get("dx"), out.get("wi"), out.get("wo"), None



# order of the FF block's backward GEMMs after dA (dX, dW_out, dW_in): which operands are still
# in the Infinity Cache when each runs.  dW_in right after dA (which it reads, 84 MB at the bench
# shape) measured best: bf16 layer 0.700 -> 0.692 ms, fp8 0.746 -> 0.739 ms over dx,wo,wi
_FF_BWD_ORDER = ["wi", "dx", "wo"]


def _ff_bwd_order(run_dx, run_wo, run_wi):
    fns = {"dx": run_dx, "wo": run_wo, "wi": run_wi}
    for k in _FF_BWD_ORDER:
        fns.pop(k)()
    for fn in fns.values():
        fn()


def ff_block_supported(x: torch.Tensor, w_in: torch.Tensor, w_out: torch.Tensor) -> bool:
    M, F = w_in.shape
    T = x.numel() // max(1, x.shape[-1])
    return (x.is_cuda and x.shape[-1] == M and tuple(w_out.shape) == (F, M) and M % 64 == 0 and F % 64 == 0
            and T % 64 == 0 and w_in.dtype == torch.float32 and w_out.dtype == torch.float32)


def ff_block(x: torch.Tensor, w_in: torch.Tensor, w_out: torch.Tensor, residual: bool) -> torch.Tensor:
    """Local fused FF block (bf16 compute): ``relu(x Win) Wout (+ x if residual)``."""
    return _FFBlock.apply(x, w_in, w_out, residual)
