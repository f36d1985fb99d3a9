"""Matmul-chain model for the FSDP / fully-sharded benchmark config (case3 at scale).

``case3_fully_sharded.py:23-46`` shards both matmul operands over the whole mesh and
lets GSPMD gather ("all gather happens", ``:57``).  At training scale that is FSDP:
every weight lives sharded over the ``data`` axis (``parallel.fsdp.fsdp_shardings``),
the partitioner all-gathers it at its use and autograd reduce-scatters its gradient.
``DenseStack`` is ``layers`` bias-free ``dim x dim`` Dense layers with ReLU between
them - a chain of sharded matmuls.  When its kernels are sharded over ``fsdp_axis``
(``bench.py --model fsdp``), layer i+1's all-gather is issued on a side HIP stream by
:class:`~..parallel.fsdp.Prefetcher` before layer i's GEMM runs, so the gather overlaps
the GEMM; autograd runs each gather's transpose (the gradient reduce-scatter) on that same
side stream, overlapping the rest of the backward pass.
"""
from __future__ import annotations

from typing import Any

import torch

from .. import dtypes as _dt
from ..nn.layers import Dense
from ..nn.module import Module
from ..ops import core
from ..sharding import NamedSharding

__all__ = ["DenseStack", "dense_stack_flops", "feed_forward_flops"]


class DenseStack(Module):
    dim: int
    layers: int = 4
    dtype: Any = torch.bfloat16
    fsdp_axis: Any = "data"

    def setup(self):
        self.blocks = [Dense(self.dim, use_bias=False, dtype=self.dtype, name=f"dense_{i}")
                       for i in range(self.layers)]

    def _prefetcher(self, w):
        """A side-stream prefetcher when ``w`` is sharded over the FSDP axis of its mesh."""
        sh = w.sharding
        if self.fsdp_axis is None or not isinstance(sh, NamedSharding):
            return None
        on_axis = any(e == self.fsdp_axis or (isinstance(e, tuple) and self.fsdp_axis in e) for e in sh.spec)
        if not on_axis or any(t.is_meta for t in w.local.values()):
            return None
        from ..parallel.fsdp import Prefetcher
        return Prefetcher(sh.mesh, self.fsdp_axis, bf16_shadows=_dt.canonicalize(self.dtype) == torch.bfloat16)

    def __call__(self, x):
        dt = _dt.canonicalize(self.dtype)
        ws = [blk.kernel_param(self.dim) for blk in self.blocks]
        pf = self._prefetcher(ws[0])
        nxt = pf.prefetch(ws[0]) if pf is not None else None
        for i in range(len(ws)):
            if pf is not None:
                w = nxt.wait()
                if i + 1 < len(ws):
                    nxt = pf.prefetch(ws[i + 1])   # in flight while this layer's GEMM runs
            else:
                w = ws[i]
            # ReLU fused into the GEMM epilogue (Dense itself has no activation)
            x = core.dense(x, [w], None, compute_dtype=dt, relu=i + 1 < len(ws))[0]
        return x


def dense_stack_flops(batch: int, seq: int, dim: int, layers: int, train: bool) -> float:
    """Matmul FLOPs; the input is not a parameter, so the first layer has no dX GEMM."""
    one = 2.0 * batch * seq * dim * dim
    return layers * one + ((2 * layers - 1) * one if train else 0.0)


def feed_forward_flops(batch: int, seq: int, dim: int, ff_dim: int, train: bool) -> float:
    """``relu(x Win) Wout`` (``case6_attention.py:36-40`` comments; case4's FC layer)."""
    one = 2.0 * batch * seq * dim * ff_dim
    return 2 * one + (3 * one if train else 0.0)
