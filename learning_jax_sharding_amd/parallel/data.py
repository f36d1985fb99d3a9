"""Data parallelism: bucketed gradient all-reduce over the replica groups, overlapped with
the backward pass.

The reference gets its data-parallel gradient sum implicitly from GSPMD when the batch is
sharded over ``data`` (``case6_attention.py:161,184,212``).  Here the partitioner's
gradient convention leaves every replica of a parameter tile with a partial gradient, and
this module sums them over each tile's replica group:

* **buckets** are filled in the order gradients become ready (autograd tensor hooks), and a
  bucket is all-reduced as soon as it holds ``bucket_bytes``.  On MI355X the whole case6
  parameter set (5.25 MB) would fit one bucket, which could never overlap; the default
  ~1 MiB cap instead launches the out-projection's gradients while the attention backward
  and the QKV weight-gradient GEMM are still running.  xGMI rings are per-link bound, so a
  few MB per collective is already past the latency knee;
* each bucket's all-reduce runs on a side comm stream (RCCL over xGMI), joined only before
  the optimizer consumes the gradients; under ``jit(capture=True)`` the collective becomes
  an asynchronous cut point of the segmented HIP-graph capture (``spmd/graphs.py``), so the
  overlap is replayed every step.

Single-process runs (host / virtual / multi-GPU in one process) use the synchronous
bucketed path of :func:`learning_jax_sharding_amd.spmd.api.reduce_replica_grads`.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..array import ShardedArray

__all__ = ["GradReducer", "default_bucket_bytes", "bucket_plan"]


def default_bucket_bytes() -> int:
    return int(float(os.environ.get("LJS_GRAD_BUCKET_MB", "1")) * (1 << 20))


def bucket_plan(sizes: Sequence[int], bucket_bytes: int) -> List[List[int]]:
    """Greedy in-order packing of byte sizes into buckets closing at ``bucket_bytes``."""
    out, cur, cb = [], [], 0
    for i, s in enumerate(sizes):
        cur.append(i)
        cb += s
        if cb >= bucket_bytes:
            out.append(cur)
            cur, cb = [], 0
    if cur:
        out.append(cur)
    return out


class GradReducer:
    """Overlapped, bucketed replica-group gradient all-reduce for one backward pass.

    ``leaves`` are the differentiated parameter arrays; ``inputs[i]`` the local torch
    leaf of ``leaves[i]`` (one local device per process in distributed runs)."""

    def __init__(self, leaves: Sequence[ShardedArray], bucket_bytes: Optional[int] = None):
        self.leaves = list(leaves)
        self.bucket_bytes = bucket_bytes or default_bucket_bytes()
        self.groups = []
        for p in self.leaves:
            ta = p.tile
            self.groups.append(tuple(tuple(ta.holders(t)) for t in sorted(set(ta.coords.values())))
            if ta.num_replicas > 1 else None)
        self.ready: Dict[int, torch.Tensor] = {}
        self.open: Dict[Tuple, List[int]] = {}
        self.open_bytes: Dict[Tuple, int] = {}
        self.launched: List[Tuple[List[int], Tuple, torch.Tensor, object]] = []

    @staticmethod
    def wanted(leaves: Sequence[ShardedArray]) -> bool:
        from ..comm.backend import get_comm
        if get_comm().kind != "dist" or os.environ.get("LJS_OVERLAP_GRAD_REDUCE", "1") == "0":
            return False
        return any(p.tile.num_replicas > 1 and any(t.is_cuda for t in p.local.values()) for p in leaves)

    # ------------------------------------------------------------------ hooks
    def attach(self, inputs: Sequence[torch.Tensor]) -> List:
        handles = []
        for i, t in enumerate(inputs):
            if self.groups[i] is None:
                continue
            handles.append(t.register_hook(lambda g, i=i: self._on_grad(i, g)))
        return handles

    def _on_grad(self, i: int, g: torch.Tensor):
        self.ready[i] = g
        key = (self.groups[i], g.dtype)
        self.open.setdefault(key, []).append(i)
        self.open_bytes[key] = self.open_bytes.get(key, 0) + g.numel() * g.element_size()
        if self.open_bytes[key] >= self.bucket_bytes:
            self._launch(key)
        return None

    def _launch(self, key):
        idxs = self.open.pop(key, [])
        self.open_bytes.pop(key, None)
        if not idxs:
            return
        groups = key[0]
        grads = [self.ready[i] for i in idxs]
        from ..comm.backend import get_comm
        from ..spmd import graphs
        me = next(iter(self.leaves[idxs[0]].local))

        def fn(grads=grads, groups=groups, me=me):
            flat = torch.cat([g.reshape(-1) for g in grads])
            return get_comm().all_reduce_({me: flat}, [tuple(g) for g in groups])[me]

        from ..spmd import plan as _plan
        _plan.record("all_reduce", groups=tuple(groups), note="grad.bucket", bytes_in=sum(
            g.numel() * g.element_size() for g in grads), overlapped=True)
        flat, handle = graphs.run_collective(fn, async_=True)
        self.launched.append((idxs, groups, flat, handle))

    # ------------------------------------------------------------------ result
    def finish(self, grads: Dict[int, Dict[int, torch.Tensor]]) -> Dict[int, Dict[int, torch.Tensor]]:
        """Launch what is left, join every bucket, return {leaf index: {dev: reduced grad}}.
        ``grads`` holds the unreduced per-leaf gradients (replica-free leaves pass through)."""
        for key in list(self.open):
            self._launch(key)
        from ..spmd import graphs
        out = dict(grads)
        for idxs, groups, flat, handle in self.launched:
            graphs.join(handle)
            off = 0
            for i in idxs:
                d, g = next(iter(grads[i].items()))
                n = g.numel()
                out[i] = {d: flat[off:off + n].view(g.shape)}
                off += n
        return out
