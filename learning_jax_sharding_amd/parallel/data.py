"""Data parallelism: bucketed gradient all-reduce over the replica groups, overlapped with
the backward pass.

The reference gets its data-parallel gradient sum implicitly from GSPMD when the batch is
sharded over ``data`` (``case6_attention.py:161,184,212``).  Here the partitioner's
gradient convention leaves every replica of a parameter tile with a partial gradient, and
this module sums them over each tile's replica group:

* **producer groups**: gradients that one kernel wrote as views of ONE buffer (the batched
  Q/K/V weight-gradient GEMM writes dWq, dWk, dWv into one ``[3, K, N]`` tensor) are held back
  until the whole buffer has arrived and then reduced as that buffer, in place - no
  concatenation, one collective instead of three;
* **buckets** are filled in the order producer groups complete (autograd tensor hooks) and
  launched as soon as one holds ``bucket_bytes`` (default 1 MiB): the output projection's
  gradients leave while the attention backward and the QKV weight-gradient GEMM still run;
* **wire dtype**: gradients travel in the parameter dtype (**f32**) by default, so a
  data-parallel step sums exactly what a single device would.  ``LJS_GRAD_COMM_DTYPE=bf16``
  is the opt-in half-bytes wire: the weight-gradient producers then also write a bf16 "twin"
  that the bucket sends (no cast kernel) - half the bytes on point-to-point xGMI rings where
  the gradient tail is exposed, at bf16 rounding of each rank's partial sum;
* each bucket's all-reduce runs on a side comm stream (RCCL over xGMI), joined only before
  the optimizer consumes the gradients.  Under ``jit(capture=True)`` a native-RCCL all-reduce
  is captured INTO the step's HIP graph (forked onto the side stream inside the capture), so
  the whole step replays as one graph; a torch-process-group one (gloo) becomes an
  asynchronous cut point of the segmented capture (``spmd/graphs.py``).  The casts on either
  side stay inside the captured graph either way.

Single-process runs (host / virtual / multi-GPU in one process) use the synchronous
bucketed path of :func:`learning_jax_sharding_amd.spmd.api.reduce_replica_grads`.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..array import ShardedArray

__all__ = ["GradReducer", "default_bucket_bytes", "bucket_plan", "comm_dtype"]


# reduced bf16 buckets are handed to the optimizer without the cast back to f32 (see finish())
_LAZY_WIRE_GRADS = os.environ.get("LJS_LAZY_WIRE_GRADS", "1") == "1"


# wire dtype of the data-parallel backward in progress (None outside one): producers of whole
# gradient buffers (the weight-grad slab combine) then also write the buffer's bf16 "twin",
# which the bucket sends instead of casting the f32 buffer itself
_ACTIVE_WIRE: Optional[torch.dtype] = None
_TWINS: Dict[int, Tuple[torch.Tensor, torch.Tensor]] = {}
# the gradient buckets of the last backward, in launch order: (bytes on the wire, dtype, groups)
# -- bench.py's comm_detail reports them
LAST_BUCKETS: List[Tuple[int, str, Tuple]] = []


def active_wire_dtype() -> Optional[torch.dtype]:
    return _ACTIVE_WIRE


def register_wire_twin(buf: torch.Tensor, twin: torch.Tensor) -> None:
    """``twin`` holds ``buf``'s values in the wire dtype (same element order)."""
    _TWINS[buf.untyped_storage().data_ptr()] = (buf, twin)


def _take_twin(flat: torch.Tensor, dtype: torch.dtype) -> Optional[torch.Tensor]:
    ent = _TWINS.pop(flat.untyped_storage().data_ptr(), None)
    if ent is None:
        return None
    buf, twin = ent
    if (twin.dtype != dtype or twin.numel() != flat.numel() or flat.storage_offset() != 0
            or buf.untyped_storage().data_ptr() != flat.untyped_storage().data_ptr()):
        return None
    return twin.reshape(-1)


def default_bucket_bytes() -> int:
    return int(float(os.environ.get("LJS_GRAD_BUCKET_MB", "1")) * (1 << 20))


def comm_dtype() -> Optional[torch.dtype]:
    """Wire dtype of f32 gradient buckets (None = as computed)."""
    v = os.environ.get("LJS_GRAD_COMM_DTYPE", "fp32").lower()
    if v in ("bf16", "bfloat16"):
        return torch.bfloat16
    if v in ("fp32", "f32", "float32", "none", ""):
        return None
    raise ValueError(f"LJS_GRAD_COMM_DTYPE={v!r}: expected bf16 or fp32")


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


def _storage_key(g: torch.Tensor) -> Tuple[int, int]:
    st = g.untyped_storage()
    return st.data_ptr(), st.nbytes()


def _covering_flat(grads: List[torch.Tensor]) -> Optional[torch.Tensor]:
    """A flat view over ``grads`` when they are contiguous views that follow each other in one
    storage, in order (a producer group, or one gradient sharing its buffer with a tail that
    belongs to another bucket, e.g. a dW with its bias gradient behind it); else None."""
    st_ptr, _ = _storage_key(grads[0])
    start = off = grads[0].storage_offset()
    for g in grads:
        if not g.is_contiguous() or _storage_key(g)[0] != st_ptr or g.storage_offset() != off:
            return None
        off += g.numel()
    return grads[0].new_empty(0).set_(grads[0].untyped_storage(), start, (off - start,), (1,))


class GradReducer:
    """Overlapped, bucketed replica-group gradient all-reduce for one backward pass.

    ``leaves`` are the differentiated parameter arrays; ``inputs[i]`` the local torch
    leaf of ``leaves[i]`` (one local device per process in distributed runs)."""

    def __init__(self, leaves: Sequence[ShardedArray], bucket_bytes: Optional[int] = None,
                 wire_dtype: Optional[torch.dtype] = "env"):
        self.leaves = list(leaves)
        self.bucket_bytes = bucket_bytes or default_bucket_bytes()
        self.wire_dtype = comm_dtype() if wire_dtype == "env" else wire_dtype
        self.groups = []
        for p in self.leaves:
            ta = p.tile
            self.groups.append(tuple(tuple(ta.holders(t)) for t in sorted(set(ta.coords.values())))
                               if ta.num_replicas > 1 else None)
        self.ready: Dict[int, torch.Tensor] = {}
        self.pending: Dict[Tuple, List[int]] = {}     # producer groups waiting for their buffer
        self.open: Dict[Tuple, List[int]] = {}
        self.open_bytes: Dict[Tuple, int] = {}
        self.launched: List[Tuple[List[int], torch.Tensor, Optional[torch.Tensor], object]] = []

    @staticmethod
    def wanted(leaves: Sequence[ShardedArray]) -> bool:
        from ..comm.backend import get_comm
        mode = os.environ.get("LJS_OVERLAP_GRAD_REDUCE", "1")
        if get_comm().kind != "dist" or mode == "0":
            return False
        # "force": also for host tensors (exercises this path in the CPU multi-process tests)
        return any(p.tile.num_replicas > 1 and (mode == "force" or any(t.is_cuda for t in p.local.values()))
                   for p in leaves)

    # ------------------------------------------------------------------ hooks
    def attach(self, inputs: Sequence[torch.Tensor]) -> List:
        global _ACTIVE_WIRE
        _ACTIVE_WIRE = self.wire_dtype
        _TWINS.clear()
        LAST_BUCKETS.clear()
        handles = []
        for i, t in enumerate(inputs):
            if self.groups[i] is None:
                continue
            handles.append(t.register_hook(lambda g, i=i: self._on_grad(i, g)))
        return handles

    def _on_grad(self, i: int, g: torch.Tensor):
        self.ready[i] = g
        skey = _storage_key(g)
        pkey = (self.groups[i], g.dtype, skey)
        members = self.pending.setdefault(pkey, [])
        members.append(i)
        seen = sum(self.ready[j].numel() * self.ready[j].element_size() for j in members)
        if seen >= skey[1]:
            # the producing buffer is complete: its views join the bucket together
            del self.pending[pkey]
            key = (self.groups[i], g.dtype)
            self.open.setdefault(key, []).extend(sorted(members, key=lambda j: self.ready[j].storage_offset()))
            self.open_bytes[key] = self.open_bytes.get(key, 0) + seen
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
        flat32 = _covering_flat(grads)
        if flat32 is None:
            parts = [g.reshape(-1) for g in grads]
            if parts[0].is_cuda and len(parts) > 1 and all(p.numel() == parts[0].numel() for p in parts):
                # equal-size gradients from separate buffers (the 2-D mesh's head-sharded Q / K / V /
                # out-projection weights): one HIP pack launch instead of torch's cat kernel
                from ..ops.hip import concat_parts
                flat32 = concat_parts(parts, 0)
            else:
                flat32 = torch.cat(parts)
        wire = None
        if self.wire_dtype is not None and flat32.dtype == torch.float32 and self.wire_dtype != flat32.dtype:
            wire = _take_twin(flat32, self.wire_dtype)
            if wire is None:
                from ..ops.hip import cast as _cast
                wire = _cast(flat32, self.wire_dtype) if flat32.is_cuda else flat32.to(self.wire_dtype)
        buf = wire if wire is not None else flat32

        def fn(buf=buf, groups=groups, me=me):
            return get_comm().all_reduce_({me: buf}, [tuple(g) for g in groups])[me]

        from ..spmd import plan as _plan
        _plan.record("all_reduce", groups=tuple(groups), note="grad.bucket", dtype=str(buf.dtype).replace("torch.", ""),
                     bytes_in=buf.numel() * buf.element_size(), overlapped=True)
        LAST_BUCKETS.append((buf.numel() * buf.element_size(), str(buf.dtype).replace("torch.", ""), tuple(groups)))
        comm = get_comm()
        _, handle = graphs.run_collective(fn, async_=True,
                                          capturable=comm.graph_safe("all_reduce", buf, [tuple(g) for g in groups]),
                                          what=f"grad bucket all_reduce {tuple(buf.shape)} {buf.dtype}")
        self.launched.append((idxs, flat32, wire, handle))

    # ------------------------------------------------------------------ result
    def finish(self, grads: Dict[int, Dict[int, torch.Tensor]]) -> Dict[int, Dict[int, torch.Tensor]]:
        """Launch what is left, join every bucket, return {leaf index: {dev: reduced grad}}.
        ``grads`` holds the unreduced per-leaf gradients (replica-free leaves pass through)."""
        global _ACTIVE_WIRE
        _ACTIVE_WIRE = None
        # the next step's input cast (if a runner registered it) fills the stream's wait for the
        # all-reduce tail below (ops/linear.py, LJS_PRECAST=join)
        from ..ops import linear as _lin
        _lin.launch_join_precasts()
        for pkey in list(self.pending):
            members = self.pending.pop(pkey)
            key = (pkey[0], pkey[1])
            self.open.setdefault(key, []).extend(members)
        for key in list(self.open):
            self._launch(key)
        _TWINS.clear()
        from ..spmd import graphs
        from ..array import LazyLocal
        out = dict(grads)
        for idxs, flat32, wire, handle in self.launched:
            graphs.join(handle)
            lazy = wire is not None and flat32.is_cuda and _LAZY_WIRE_GRADS
            if wire is not None and not lazy:
                # back to the gradients' dtype inside the captured segment after the join
                from ..ops.hip import cast_into as _cast_into
                if flat32.is_cuda:
                    _cast_into(wire, flat32)
                else:
                    flat32.copy_(wire)
            cast_once = None
            if lazy:
                # the reduced bucket stays in the wire dtype: the fused Adam reads bf16 gradients
                # directly (LazyLocal.raw), and the f32 view is produced -- by one cast of the whole
                # bucket -- only if something else reads the gradient values
                done = []

                def cast_once(wire=wire, flat32=flat32, done=done):
                    if not done:
                        from ..ops.hip import cast_into as _cast_into
                        _cast_into(wire, flat32)
                        done.append(True)
            off = 0
            for i in idxs:
                d, g = next(iter(grads[i].items()))
                n = g.numel()
                if lazy:
                    ll = LazyLocal(lambda d=d, o=off, n=n, sh=g.shape, c=cast_once, f=flat32:
                                   (c(), {d: f[o:o + n].view(sh)})[1])
                    ll.raw = {d: wire[off:off + n].view(g.shape)}
                    out[i] = ll
                else:
                    out[i] = {d: flat32[off:off + n].view(g.shape)}
                off += n
        return out
