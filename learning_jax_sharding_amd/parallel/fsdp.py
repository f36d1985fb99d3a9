"""Fully-sharded data parallelism (ZeRO-3 style) with prefetched parameter all-gathers.

Reference behaviour: ``case5_attention_dense.py:109-112`` maps the ``embed`` logical axis
onto ``data``, so every weight lives sharded over the data-parallel axis and GSPMD gathers
it at use and reduce-scatters its gradient; ``case3_fully_sharded.py:23-46`` is the bare
matmul form (both operands fully sharded, "all gather happens", ``:57``).

On MI355X the gathers and the gradient reduce-scatters run on a side HIP stream:

* :func:`fsdp_shardings` picks, per parameter, the largest dim divisible by the axis size;
* :class:`Prefetcher` issues the all-gathers of the NEXT layer's parameters on a side
  stream while the current layer computes, and hands back arrays already replicated over
  the axis (the partitioner then inserts no gather of its own).  The gathers are the
  framework's differentiable collectives, so autograd runs their transposes - the
  gradient reduce-scatters - on that same side stream, overlapping the rest of the
  backward pass;
* :func:`gathered` is the synchronous form (gather on the side stream, wait, return).

With 288 GB of HBM per GPU the prefetch depth is a latency knob, not a memory one: one
layer ahead already hides an xGMI gather behind a layer's GEMMs.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

import torch

from ..array import ShardedArray
from ..mesh import Mesh, current_mesh
from ..sharding import NamedSharding, PartitionSpec as P
from ..spmd.reshard import reshard_tile
from ..utils import tree as T

__all__ = ["fsdp_shardings", "shard_params", "Prefetcher", "gathered"]


def _is_arr(x):
    return isinstance(x, ShardedArray)


def fsdp_shardings(params, mesh: Mesh, axis: str = "data", min_elements: int = 1024):
    """NamedShardings placing each parameter's largest axis-divisible dim on ``axis``
    (small or indivisible params stay replicated)."""
    n = mesh.shape[axis]

    def pick(p):
        shape = tuple(p.shape)
        spec = [None] * len(shape)
        if int(torch.tensor(shape).prod()) >= min_elements if shape else False:
            dims = sorted(range(len(shape)), key=lambda d: -shape[d])
            for d in dims:
                if shape[d] % n == 0:
                    spec[d] = axis
                    break
        return NamedSharding(mesh, P(*spec))
    return T.tree_map(pick, params, is_leaf=lambda x: hasattr(x, "shape"))


def shard_params(params, mesh: Mesh, axis: str = "data"):
    """Place a parameter tree FSDP-style over ``axis``."""
    from ..array import device_put
    return device_put(params, fsdp_shardings(params, mesh, axis))


class _Handle:
    def __init__(self, tree, event: Optional[torch.cuda.Event], stream):
        self._tree = tree
        self._event = event
        self._stream = stream
        self._waited = False

    def tree(self):
        """The gathered tree WITHOUT ordering the current stream after the gathers (the consumer
        must call :meth:`wait` before any kernel reads it - ops.linear.defer_wait)."""
        return self._tree

    def wait(self):
        """The gathered tree, ordered after the side-stream gathers on the current stream."""
        if self._waited:
            return self._tree
        self._waited = True
        if self._event is not None:
            cur = torch.cuda.current_stream()
            cur.wait_event(self._event)
            from ..ops import shadow as _shadow
            for leaf in T.tree_leaves(self._tree, is_leaf=_is_arr):
                if _is_arr(leaf):
                    for t in leaf.local.values():
                        if t.is_cuda:
                            t.record_stream(cur)
                            if t.dim() == 2 and _shadow.is_proxy(t):
                                # a gathered-weight proxy: its data is the bf16 buffer the side
                                # stream allocated (kept by the shadow registry)
                                for buf in _shadow.kinds_of(t).values():
                                    buf.record_stream(cur)
        return self._tree


class Prefetcher:
    """Gathers FSDP-sharded parameters over ``axis`` on a side stream ahead of use."""

    def __init__(self, mesh: Optional[Mesh] = None, axis: str = "data", bf16_shadows: bool = False):
        """``bf16_shadows``: the consumers are bf16 GEMMs - 2-D f32 weights are gathered as their
        shards' bf16 shadows (parallel/weight_gather.py: half the bytes, no cast kernel)."""
        self.mesh = mesh or current_mesh()
        if self.mesh is None:
            raise ValueError("Prefetcher needs a mesh")
        self.axis = axis
        self.bf16_shadows = bf16_shadows
        self._streams: Dict[int, torch.cuda.Stream] = {}

    def _gather_leaf(self, p: ShardedArray) -> ShardedArray:
        """Unshard the dims that live on ``axis`` (other mesh axes keep their tiling)."""
        ta = p.tile
        sh = p.sharding
        if isinstance(sh, NamedSharding):
            spec = tuple(sh.spec) + (None,) * (p.ndim - len(sh.spec))
            dims = [d for d, e in enumerate(spec)
                    if e == self.axis or (isinstance(e, tuple) and self.axis in e)]
        else:
            dims = [d for d in range(p.ndim) if ta.tile_shape[d] > 1]
        if not dims:
            return p
        dst = ta.unshard(dims)
        if self.bf16_shadows:
            from . import weight_gather as _wg
            gdim = _wg.eligible([p], dst)
            if gdim is not None:
                return _wg.gather_bf16([p], dst, gdim, note="fsdp.prefetch")[0]
        return reshard_tile(p, dst, note="fsdp.prefetch")

    def prefetch_joint(self, ws) -> _Handle:
        """Gather same-sharded 2-D weights (e.g. Q/K/V) as ONE collective of their stacked bf16
        shadows on the side stream (per weight when that does not apply)."""
        ws = list(ws)
        w0 = ws[0]
        dims = self._dims(w0)
        if not dims or any(w.tile != w0.tile or tuple(w.shape) != tuple(w0.shape) for w in ws):
            return self.prefetch(ws)
        dst = w0.tile.unshard(dims)
        from . import weight_gather as _wg
        gdim = _wg.eligible(ws, dst) if self.bf16_shadows else None
        if gdim is None:
            return self.prefetch(ws)
        devs = sorted({t.device.index for w in ws for t in w.local.values() if t.is_cuda})
        dev = devs[0]
        from ..spmd import graphs as _graphs
        if not _graphs.forks_ok():   # (a segmented capture cut at these gathers: no fork)
            return _Handle(_wg.gather_bf16(ws, dst, gdim, note="prefetch.joint"), None, None)
        s = self._streams.get(dev)
        if s is None:
            s = self._streams[dev] = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            out = _wg.gather_bf16(ws, dst, gdim, note="prefetch.joint")
            ev = torch.cuda.Event()
            ev.record(s)
        return _Handle(out, ev, s)

    def _dims(self, p: ShardedArray):
        sh = p.sharding
        if isinstance(sh, NamedSharding):
            spec = tuple(sh.spec) + (None,) * (p.ndim - len(sh.spec))
            return [d for d, e in enumerate(spec) if e == self.axis or (isinstance(e, tuple) and self.axis in e)]
        return [d for d in range(p.ndim) if p.tile.tile_shape[d] > 1]

    def prefetch(self, tree: Any) -> _Handle:
        leaves = [l for l in T.tree_leaves(tree, is_leaf=_is_arr) if _is_arr(l)]
        devs = sorted({t.device.index for l in leaves for t in l.local.values() if t.is_cuda})
        from ..spmd import graphs as _graphs
        if not devs or not _graphs.forks_ok():   # (host arrays, or a capture cut at the gathers)
            return _Handle(T.tree_map(lambda l: self._gather_leaf(l) if _is_arr(l) else l, tree, is_leaf=_is_arr),
                           None, None)
        dev = devs[0]
        s = self._streams.get(dev)
        if s is None:
            s = self._streams[dev] = torch.cuda.Stream(device=dev)
        cur = torch.cuda.current_stream(dev)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            out = T.tree_map(lambda l: self._gather_leaf(l) if _is_arr(l) else l, tree, is_leaf=_is_arr)
            ev = torch.cuda.Event()
            ev.record(s)
        return _Handle(out, ev, s)


def gathered(tree: Any, mesh: Optional[Mesh] = None, axis: str = "data"):
    """Synchronous convenience: all-gather an FSDP-sharded tree (on the side stream)."""
    return Prefetcher(mesh, axis).prefetch(tree).wait()
