"""The case6 multi-head self-attention block (the north-star workload).

Same parameters, logical axes and sharding constraints as
``FlaxAttention`` in ``case6_attention.py:42-143``:

* ``to_q``/``to_k``/``to_v``: Dense(inner_dim, no bias), kernel axes ``('embed','heads')``
  (``case6_attention.py:56-82``);
* ``to_out_0``: Dense(query_dim, bias), kernel axes ``('heads','embed')``
  (``case6_attention.py:83-90``);
* constraints ``('batch','embed',None)`` on q/k/v (``:105-107``), the head split
  (``:109-116``), ``('batch','kv','heads')`` after merging heads (``:137``) and
  ``('batch','embed')`` on the output (``:141``).

MI355X design: the three projections run as ONE batched MFMA GEMM over the
concatenated kernels (``fused_qkv``), and QKᵀ → scale → softmax → P·V is one
flash-style HIP kernel (``impl="fused"``).  ``impl="einsum"`` runs the
reference's literal einsum/softmax formulation (used by the parity tests).
"""
from __future__ import annotations

import contextlib
import os
from typing import Any, Optional

import torch

from .. import dtypes as _dt
from ..array import ShardedArray
from ..nn import initializers as init
from ..nn.layers import Dense, Dropout
from ..nn.module import Module
from ..nn.partitioning import with_logical_constraint, with_logical_partitioning
from ..ops import core

__all__ = ["MultiHeadAttention", "attention_block_flops"]


class MultiHeadAttention(Module):
    query_dim: int
    heads: int = 8
    dim_head: int = 64
    dropout: float = 0.0
    dtype: Any = torch.bfloat16
    impl: str = "fused"            # "fused" (HIP flash attention) | "einsum" (reference formulation)
    fused_qkv: bool = True
    kernel_axes_in: tuple = ("embed", "heads")
    kernel_axes_out: tuple = ("heads", "embed")
    verbose: bool = False

    def setup(self):
        inner_dim = self.dim_head * self.heads
        self.scale = self.dim_head ** -0.5
        qkv_init = with_logical_partitioning(init.lecun_normal(), self.kernel_axes_in)
        self.query = Dense(inner_dim, kernel_init=qkv_init, use_bias=False, dtype=self.dtype, name="to_q")
        self.key = Dense(inner_dim, kernel_init=qkv_init, use_bias=False, dtype=self.dtype, name="to_k")
        self.value = Dense(inner_dim, kernel_init=qkv_init, use_bias=False, dtype=self.dtype, name="to_v")
        self.proj_attn = Dense(self.query_dim,
                               kernel_init=with_logical_partitioning(init.lecun_normal(), self.kernel_axes_out),
                               dtype=self.dtype, name="to_out_0")
        self.dropout_layer = Dropout(rate=self.dropout)

    def _prefetch_out_kernel(self, x: ShardedArray, dt):
        wo = self.proj_attn.kernel_param(self.dim_head * self.heads)
        if any(t.is_meta or not t.is_cuda for t in wo.local.values()):
            return None
        axis = _fsdp_axis(wo, x)
        if axis is None:
            return None
        from ..parallel.fsdp import Prefetcher
        return Prefetcher(wo.sharding.mesh, axis, bf16_shadows=dt == torch.bfloat16).prefetch([wo])

    def _prefetch_qkv(self, x: ShardedArray, ws, dt):
        from ..sharding import NamedSharding
        w0 = ws[0]
        if dt != torch.bfloat16 or any(t.is_meta or not t.is_cuda for w in ws for t in w.local.values()):
            return None
        if not qkv_prefetch_wanted(w0):
            return None
        sh, xs = w0.sharding, x.sharding
        if not isinstance(sh, NamedSharding) or not isinstance(xs, NamedSharding) or not sh.spec:
            return None
        if any(w.sharding != sh for w in ws):
            return None
        axis = sh.spec[0]
        if not isinstance(axis, str) or sh.mesh.shape[axis] < 2 or (len(sh.spec) > 1 and sh.spec[1] is not None):
            return None
        xspec = tuple(xs.spec) + (None,) * (x.ndim - len(xs.spec))
        if xspec[-1] is not None:
            return None
        from ..parallel.fsdp import Prefetcher
        return Prefetcher(sh.mesh, axis, bf16_shadows=True).prefetch_joint(ws)

    def _log(self, *a):
        if self.verbose:
            print(*a)

    def __call__(self, hidden_states: ShardedArray, context: Optional[ShardedArray] = None,
                 deterministic: bool = True, residual: Optional[ShardedArray] = None) -> ShardedArray:
        """``residual`` (the block's input, for a skip connection): returns
        ``residual + attention(...)`` in the compute dtype, the add fused into the output
        projection's GEMM epilogue when dropout is the identity."""
        self_attn = context is None
        context = hidden_states if context is None else context
        self._log("context.shape: ", context.shape)
        dt = _dt.canonicalize(self.dtype)
        # FSDP rules (case5_attention_dense.py:109-112: embed -> data) shard the out projection's
        # kernel over the batch axis: gather it on a side stream NOW, while the QKV projection and
        # the attention run, instead of at its use (parallel/fsdp.py Prefetcher, bf16 shadows)
        wo_pf = self._prefetch_out_kernel(hidden_states, dt)
        if self.fused_qkv and self_attn:
            m = hidden_states.shape[-1]
            wq = self.query.kernel_param(m)
            wk = self.key.kernel_param(m)
            wv = self.value.kernel_param(m)
            # Q/K/V kernels sharded over their input features (the reference's 2-D rules: embed
            # -> model) while the activation's features are whole: their one stacked bf16 gather
            # runs on a side stream, and the projection GEMM waits for it only after queueing
            # the activation's cast pass (ops/linear.defer_wait)
            qkv_pf = self._prefetch_qkv(hidden_states, [wq, wk, wv], dt)
            if qkv_pf is not None:
                from ..ops import linear as _lin
                _lin.defer_wait(qkv_pf)
                ws = qkv_pf.tree()
            else:
                ws = [wq, wk, wv]
            # the attention forward rides in the projection kernel when every device holds whole
            # sequences and all heads (ops/linear.attention_next: single device / data parallel)
            from ..ops import linear as _lin
            hint = (self.impl == "fused" and qkv_pf is None and hidden_states.ndim == 3
                    and tuple(hidden_states.tile.tile_shape[1:]) == (1, 1)
                    and all(tuple(w.tile.tile_shape) == (1, 1) for w in (wq, wk, wv)))
            with (_lin.attention_next(self.heads, self.dim_head, self.scale) if hint else contextlib.nullcontext()):
                query_proj, key_proj, value_proj = core.dense(hidden_states, ws, None, compute_dtype=dt)
            if qkv_pf is not None:
                qkv_pf.wait()
        else:
            query_proj = self.query(hidden_states)
            key_proj = self.key(context)
            value_proj = self.value(context)
        self._log("query_proj.shape: ", query_proj.shape)

        # (batch, seq, heads*head_dim); the head split is metadata-only because heads is replicated
        query_proj = with_logical_constraint(query_proj, ("batch", "embed", None))
        key_proj = with_logical_constraint(key_proj, ("batch", "embed", None))
        value_proj = with_logical_constraint(value_proj, ("batch", "embed", None))

        b = hidden_states.shape[0]
        q = core.reshape(query_proj, (b, -1, self.heads, self.dim_head))
        k = core.reshape(key_proj, (b, -1, self.heads, self.dim_head))
        v = core.reshape(value_proj, (b, -1, self.heads, self.dim_head))
        q = with_logical_constraint(q, ("batch", "embed", None, None))
        k = with_logical_constraint(k, ("batch", "embed", None, None))
        v = with_logical_constraint(v, ("batch", "embed", None, None))
        self._log("query_states.shape: ", q.shape)

        if self.impl == "fused":
            hidden = core.dot_product_attention(q, k, v, self.scale)
        else:
            qf = core.convert(q, torch.float32)
            kf = core.convert(k, torch.float32)
            scores = core.einsum("b t n h, b f n h -> b n f t", kf, qf)
            scores = core.binary("mul", scores, self.scale)
            probs = core.softmax(scores, axis=-1)
            probs = core.convert(probs, dt)
            hidden = core.einsum("b n f t, b t n h -> b f n h", probs, v)
        hidden = core.reshape(hidden, (b, -1, self.heads * self.dim_head))
        hidden = with_logical_constraint(hidden, ("batch", "kv", "heads"))
        drop_id = deterministic or self.dropout == 0.0
        wo = wo_pf.wait()[0] if wo_pf is not None else None
        if residual is not None and drop_id:
            hidden = self.proj_attn(hidden, residual=residual, kernel=wo)
            return with_logical_constraint(hidden, ("batch", "embed"))
        hidden = self.proj_attn(hidden, kernel=wo)
        hidden = with_logical_constraint(hidden, ("batch", "embed"))
        hidden = self.dropout_layer(hidden, deterministic=deterministic)
        if residual is not None:
            hidden = core.binary("add", core.convert(residual, dt), hidden)
        return hidden


# Measured: the gather overlaps the activation cast (profiles/r3k_v2x2_prefetch_overlap.md), but
# the side-stream branch costs more than it hides when the "gather" moves no bytes between GPUs:
# 2-D rehearsal 0.3378-0.3404 vs 0.3165-0.3172 ms, 4 virtual devices 1.79-1.80 vs 1.62 ms
# (gpurun_out/r3k).  Over xGMI it is a real transfer worth hiding.  LJS_QKV_PREFETCH: "1" on,
# "0" off, "auto" (default): on exactly when the gather crosses between distinct GPUs.
_QKV_PREFETCH = os.environ.get("LJS_QKV_PREFETCH", "auto").lower()


def qkv_prefetch_wanted(w: ShardedArray) -> bool:
    """Whether the Q/K/V weight gather of ``w``'s layout is prefetched on a side stream."""
    if _QKV_PREFETCH in ("0", "1"):
        return _QKV_PREFETCH == "1"
    from ..comm.backend import get_comm
    c = get_comm()
    if c.kind == "dist":
        return c.real_transfers()
    return c.real_transfers([t.device for t in w.local.values()])


def _fsdp_axis(w: ShardedArray, x: ShardedArray):
    """The mesh axis sharding both ``w`` and ``x``'s batch dim (the FSDP pattern), else None."""
    from ..sharding import NamedSharding
    ws, xs = w.sharding, x.sharding
    if not isinstance(ws, NamedSharding) or not isinstance(xs, NamedSharding) or not xs.spec:
        return None
    b = xs.spec[0]
    b_axes = set(b) if isinstance(b, tuple) else ({b} if b else set())
    for e in ws.spec:
        for a in (e if isinstance(e, tuple) else (e,)):
            if a is not None and a in b_axes and ws.mesh.shape[a] > 1:
                return a
    return None


def attention_block_flops(batch: int, seq: int, dim: int, heads: int, dim_head: int, train: bool) -> float:
    """Matmul FLOPs of the case6 block: fwd 6.442 GFLOP at B=8,S=256,M=640; train 15.30."""
    t = batch * seq
    inner = heads * dim_head
    qkv = 3 * 2 * t * dim * inner
    qk = 2 * batch * heads * seq * seq * dim_head
    pv = qk
    out = 2 * t * inner * dim
    fwd = qkv + qk + pv + out
    if not train:
        return float(fwd)
    # backward: dWo + dh (2 out-proj GEMMs), attention bwd (dV, dP, dQ, dK = 4 seq^2 GEMMs), dWqkv (no dx)
    bwd = 2 * out + 4 * qk + qkv
    return float(fwd + bwd)
