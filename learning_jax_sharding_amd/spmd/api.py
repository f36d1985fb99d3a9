"""``jit`` / ``grad`` / ``value_and_grad`` / ``eval_shape``.

* ``jit(f, in_shardings, out_shardings, static_argnums, donate_argnums)``
  (``case6_attention.py:192-194,206-207,229-230``): reshard inputs to
  ``in_shardings``, run ``f`` through the eager SPMD partitioner
  (:mod:`..ops.core`), reshard outputs to ``out_shardings``.  Instead of a
  tracing compiler, the MI355X fast path is a **HIP graph**: with
  ``capture=True`` (or ``LJS_JIT_GRAPH=1``) the second call with a given
  signature is captured into a ``torch.cuda.CUDAGraph`` (hipGraph on ROCm) and
  every later call is one graph replay - no Python, no partitioning, no
  per-kernel launch cost.  Outputs of a captured function live in the graph's
  static buffers and are overwritten by the next call (the same contract as
  donated buffers).
* ``grad`` (``case6_attention.py:212``): reverse mode through torch autograd
  on the per-device shards.  Collectives are differentiable with transposed
  collectives (:mod:`..comm.collectives`).  The per-device cotangents of a
  parameter are partial; they are summed over each tile's replica group with
  one bucketed all-reduce per replica-group pattern - this *is* the data
  parallel gradient all-reduce, derived from the shardings.
* ``eval_shape`` (``case6_attention.py:189``): run ``f`` on meta tensors.
"""
from __future__ import annotations

import os
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import torch

from ..array import LazyLocal, ShapeDtypeStruct, ShardedArray, device_put
from ..comm import collectives as C
from ..sharding.shardings import Sharding, SingleDeviceSharding
from ..sharding.tile import TileAssignment
from ..utils import tree as T
from . import plan as _plan
from . import state as _state
from .reshard import reshard

__all__ = ["jit", "grad", "value_and_grad", "eval_shape", "Jitted", "reduce_replica_grads"]


def _is_arraylike(x) -> bool:
    import numpy as np
    return isinstance(x, (ShardedArray, torch.Tensor, np.ndarray))


def _apply_shardings(tree, shardings):
    """Reshard / place every array leaf of ``tree`` per the (prefix) tree ``shardings``."""
    if shardings is None:
        return tree

    def place(x, s):
        if s is None or not _is_arraylike(x):
            return x
        if isinstance(x, ShardedArray):
            return reshard(x, s)
        return device_put(x, s)

    return T.tree_map(place, tree, shardings, is_leaf=lambda x: isinstance(x, (ShardedArray, ShapeDtypeStruct)))


def _leaf_is_array(x):
    return isinstance(x, ShardedArray)


class Lowered:
    def __init__(self, plan: _plan.PlanRecorder):
        self.plan = plan

    def as_text(self) -> str:
        return self.plan.as_text()

    def compile(self):
        return self


class _Captured:
    """A hipGraph of one call signature: static inputs, static outputs."""

    def __init__(self, graph, in_leaves, out_tree, aliased):
        self.graph = graph
        self.in_leaves = in_leaves  # list of ShardedArray (static buffers)
        self.out_tree = out_tree
        self.aliased = aliased      # per leaf: the caller's own buffers (read-only in the graph)


def _force_lazy(tree):
    """Materialise every pending :class:`LazyLocal` among ``tree``'s arrays (returns ``tree``)."""
    for l in T.tree_leaves(tree, is_leaf=_leaf_is_array):
        if isinstance(l, ShardedArray) and isinstance(l.local, LazyLocal) and l.local.pending:
            l.local._force()
    return tree


class Jitted:
    def __init__(self, fun: Callable, in_shardings=None, out_shardings=None, static_argnums=(),
                 donate_argnums=(), capture: Optional[bool] = None, warmup_calls: int = 1):
        self.fun = fun
        self.in_shardings = in_shardings
        self.out_shardings = out_shardings
        self.static_argnums = (static_argnums,) if isinstance(static_argnums, int) else tuple(static_argnums)
        self.donate_argnums = (donate_argnums,) if isinstance(donate_argnums, int) else tuple(donate_argnums)
        if capture is None:
            capture = os.environ.get("LJS_JIT_GRAPH", "0") == "1"
        self.capture = capture
        self.warmup_calls = warmup_calls
        self._calls: Dict[Any, int] = {}
        self._graphs: Dict[Any, _Captured] = {}
        self._fast = None   # (args of the last replay, its capture, its input copies)
        self._md_failed = set()   # signatures whose multi-GPU capture failed (run eagerly)
        self.__wrapped__ = fun

    # ------------------------------------------------------------------ helpers
    def _split(self, args):
        dyn, static = [], []
        for i, a in enumerate(args):
            (static if i in self.static_argnums else dyn).append((i, a))
        return dyn, static

    def _signature(self, dyn, static):
        leaves, td = T.tree_flatten([a for _, a in dyn], is_leaf=_leaf_is_array)
        sig = []
        for l in leaves:
            if isinstance(l, ShardedArray):
                sig.append(("A", l.shape, l.dtype, l.tile))
            else:
                sig.append(("O", type(l).__name__, repr(l) if not _is_arraylike(l) else getattr(l, "shape", None)))
        skey = []
        for i, a in static:
            try:
                hash(a)
                skey.append((i, a))
            except TypeError:
                skey.append((i, id(a)))
        return (td, tuple(sig), tuple(skey))

    def _run(self, args, kwargs):
        dyn, static = self._split(args)
        dyn_vals = [a for _, a in dyn]
        if self.in_shardings is not None:
            ins = self.in_shardings
            if not isinstance(ins, (tuple, list)) or len(dyn_vals) == 1 and not isinstance(ins, tuple):
                ins = (ins,) if len(dyn_vals) == 1 else ins
            dyn_vals = list(_apply_shardings(tuple(dyn_vals), tuple(ins)))
        full = list(args)
        for (i, _), v in zip(dyn, dyn_vals):
            full[i] = v
        donated = set()
        for i in self.donate_argnums:
            for l in T.tree_leaves(full[i], is_leaf=_leaf_is_array):
                if isinstance(l, ShardedArray):
                    donated.update(id(t) for t in l.local.values())
        placed = self._placement(full)
        with _state.donating(donated), _state.placement(placed), _state.user_code():
            out = self.fun(*full, **kwargs)
        if self.out_shardings is not None:
            out = _apply_shardings(out, self.out_shardings)
        return out, full

    def _placement(self, full):
        """The jit's device set: where arrays created inside the function are placed."""
        from ..sharding.shardings import NamedSharding, ReplicatedSharding
        cands = []
        for tree in (self.in_shardings, self.out_shardings):
            if tree is not None:
                cands += [s for s in T.tree_leaves(tree, is_leaf=lambda x: isinstance(x, Sharding))
                          if isinstance(s, NamedSharding)]
        for a in full:
            cands += [l.sharding for l in T.tree_leaves(a, is_leaf=_leaf_is_array)
                      if isinstance(l, ShardedArray) and isinstance(l.sharding, NamedSharding)]
        if not cands:
            return None
        return ReplicatedSharding(tuple(cands[0].mesh.devices.flat))

    # ------------------------------------------------------------------ call
    def __call__(self, *args, **kwargs):
        fast = self._fast
        if fast is not None and not kwargs and len(args) == len(fast[0]) and all(
                a is b for a, b in zip(args, fast[0])):
            # the very same argument objects as the last replay (e.g. a train loop feeding the
            # state the graph returned): same leaves, same copies - skip signature and checks.
            # The previous args stay referenced, so their ids cannot be reused meanwhile.
            cap, copies = fast[1], fast[2]
            for t, s in copies:
                t.copy_(s)
            cap.graph.replay()
            return cap.out_tree
        dyn, static = self._split(args)
        sig = self._signature(dyn, static)
        if not self.capture or kwargs or not torch.cuda.is_available() or (
                _spans_gpus() and (not _MULTI_GPU_CAPTURE or sig in self._md_failed)):
            # Python side effects (print) run once per signature, as at JAX trace time
            n = self._calls.get(sig, 0)
            self._calls[sig] = n + 1
            if n == 0 or os.environ.get("LJS_TRACE_PRINTS") == "always":
                return self._run(args, kwargs)[0]
            import contextlib
            import io
            with contextlib.redirect_stdout(io.StringIO()):
                return self._run(args, kwargs)[0]
        cap = self._graphs.get(sig)
        if cap is not None:
            return self._replay(cap, args, sig)
        n = self._calls.get(sig, 0)
        self._calls[sig] = n + 1
        if n < self.warmup_calls:
            return self._run(args, kwargs)[0]
        return self._capture(sig, args)

    def _capture(self, sig, args, alias: bool = True):
        """Capture one call into a hipGraph.  Static inputs: donated buffers as they are (the
        graph updates them in place; their bf16 weight shadows stay valid); other inputs are
        aliased too (the graph only reads them), so a caller that passes the same arrays again
        costs no copy.  A later call with different buffers re-captures once with private
        static copies, into which every further call's inputs are copied."""
        dyn, static = self._split(args)
        full = list(args)
        in_leaves, aliased = [], []
        for i, a in dyn:
            donated = i in self.donate_argnums

            def cp(x, donated=donated):
                if isinstance(x, ShardedArray):
                    keep = donated or alias
                    y = x if keep else ShardedArray(x.shape, x.dtype, x.sharding,
                                                    {d: t.detach().clone() for d, t in x.local.items()})
                    in_leaves.append(y)
                    aliased.append(keep and not donated)
                    return y
                return x
            full[i] = T.tree_map(cp, a, is_leaf=_leaf_is_array)
        # lazy outputs (an unread loss, uncombined weight gradients) are forced INSIDE the
        # capture: a thunk run after it would be eager, cached, and stale on every later replay
        if _spans_gpus():
            # single controller over several GPUs: ONE graph with a branch per device
            from .graphs import MultiDeviceGraph
            g = MultiDeviceGraph(_gpu_indices())
            try:
                out = g.capture(lambda: _force_lazy(self._run(tuple(full), {})[0]))
            except Exception as e:   # (e.g. a runtime without multi-device graphs) -> eager
                import warnings
                warnings.warn(f"multi-GPU graph capture failed ({e!r}); running this step eagerly")
                g.release()
                self._md_failed.add(sig)
                torch.cuda.synchronize()
                return self._run(args, {})[0]
        else:
            # one HIP graph per stretch between cross-process collectives (spmd/graphs.py)
            from .graphs import SegmentedGraph
            g = SegmentedGraph()
            out = g.capture(lambda: _force_lazy(self._run(tuple(full), {})[0]))
        cap = _Captured(g, in_leaves, out, aliased)
        self._graphs[sig] = cap
        return self._replay(cap, args, sig)

    def _replay(self, cap: _Captured, args, sig=None):
        dyn, _ = self._split(args)
        leaves = [l for _, a in dyn for l in T.tree_leaves(a, is_leaf=_leaf_is_array) if isinstance(l, ShardedArray)]
        copies = []
        for src, dst, al in zip(leaves, cap.in_leaves, cap.aliased):
            for d, t in dst.local.items():
                s = src.local[d]
                if s.data_ptr() != t.data_ptr() or s.stride() != t.stride():
                    if al:  # never write into a caller's buffer: re-capture with private inputs
                        if sig is None:
                            sig = self._signature(*self._split(args))
                        return self._capture(sig, args, alias=False)
                    copies.append((t, s))
        if copies and _REPLAY_TRACE and not getattr(cap, "_traced", False):
            cap._traced = True
            import sys
            print(f"[ljs replay] {len(copies)} input copies per replay: "
                  + ", ".join(f"{s.dtype}{list(s.shape)}" for _, s in copies[:40]), file=sys.stderr)
        for t, s in copies:
            t.copy_(s)
        cap.graph.replay()
        self._fast = (tuple(args), cap, copies)
        return cap.out_tree

    def lower(self, *args, **kwargs) -> Lowered:
        with _plan.record_plan() as rec:
            self._run(args, kwargs)
        return Lowered(rec)


def jit(fun: Optional[Callable] = None, *, in_shardings=None, out_shardings=None, static_argnums=(),
        donate_argnums=(), capture: Optional[bool] = None, warmup_calls: int = 1):
    if fun is None:
        return lambda f: jit(f, in_shardings=in_shardings, out_shardings=out_shardings,
                             static_argnums=static_argnums, donate_argnums=donate_argnums,
                             capture=capture, warmup_calls=warmup_calls)
    return Jitted(fun, in_shardings, out_shardings, static_argnums, donate_argnums, capture, warmup_calls)


# ----------------------------------------------------------------------------- grad
def _fresh_leaf(x: ShardedArray) -> ShardedArray:
    loc = {}
    for d, t in x.local.items():
        if t.dtype.is_floating_point:
            leaf = t.detach().requires_grad_(True)
            leaf._ljs_base = t      # the persistent parameter (owner of its bf16 shadows, ops/shadow.py)
            loc[d] = leaf
        else:
            loc[d] = t
    return ShardedArray(x.shape, x.dtype, x.sharding, loc)


def reduce_replica_grads(pairs: List[Tuple[ShardedArray, Dict[int, torch.Tensor]]],
                         bucket_bytes: int = 256 << 20) -> List[Dict[int, torch.Tensor]]:
    """Sum partial per-device gradients over each tile's replica group (bucketed all-reduce).

    ``pairs`` = [(param, {dev: partial grad})].  Params whose replica groups
    coincide share flat buckets (one all-reduce per bucket).  On MI355X the
    bucket size defaults to 256 MB: with 288 GB of HBM per GPU there is no
    memory reason to split, and fewer, larger RCCL calls amortise latency on
    point-to-point xGMI rings.
    """
    from ..parallel import data as _data
    _data.LAST_BUCKETS.clear()
    out: List[Optional[Dict[int, torch.Tensor]]] = [None] * len(pairs)
    buckets: Dict[Tuple, List[int]] = {}
    for i, (p, g) in enumerate(pairs):
        ta = p.tile
        if ta.num_replicas == 1:
            out[i] = g
            continue
        groups = tuple(tuple(ta.holders(t)) for t in sorted(set(ta.coords.values())))
        key = (groups, next(iter(g.values())).dtype if g else None)
        buckets.setdefault(key, []).append(i)
    for (groups, dt), idxs in buckets.items():
        # split into size-capped buckets (in parameter order)
        cur: List[int] = []
        cur_bytes = 0
        chunks: List[List[int]] = []
        for i in idxs:
            nb = max(t.numel() * t.element_size() for t in pairs[i][1].values()) if pairs[i][1] else 0
            if cur and cur_bytes + nb > bucket_bytes:
                chunks.append(cur)
                cur, cur_bytes = [], 0
            cur.append(i)
            cur_bytes += nb
        if cur:
            chunks.append(cur)
        for chunk in chunks:
            devs = list(pairs[chunk[0]][1].keys())
            flat = {d: torch.cat([pairs[i][1][d].reshape(-1) for i in chunk]) for d in devs}
            f0 = next(iter(flat.values()))
            _data.LAST_BUCKETS.append((f0.numel() * f0.element_size(), str(f0.dtype).replace("torch.", ""),
                                       tuple(groups)))
            red = C.all_reduce(flat, groups, note="grad.replica_sum")
            for d in devs:
                off = 0
                for i in chunk:
                    t = pairs[i][1][d]
                    n = t.numel()
                    if out[i] is None:
                        out[i] = {}
                    out[i][d] = red[d][off:off + n].view(t.shape)
                    off += n
    return out  # type: ignore


def _multi_process() -> bool:
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _gpu_indices() -> List[int]:
    from ..runtime.devices import local_devices
    return sorted({d.torch_device.index for d in local_devices() if d.platform == "gpu"})


def _spans_gpus() -> bool:
    """Single-controller run over several physical GPUs: captured as ONE multi-device graph
    (spmd/graphs.py MultiDeviceGraph; its collectives are the grouped single-controller RCCL
    calls of comm/native.py, graph nodes on every device's branch).  One process per GPU
    (torchrun) captures each rank's step as usual."""
    return len(_gpu_indices()) > 1


# Single-controller multi-GPU steps run eagerly unless LJS_MULTI_GPU_CAPTURE=1 (then captured as
# one MultiDeviceGraph; the capture falls back to eager by itself if the runtime refuses it).
# Opt-in until a cross-device capture has run on multi-GPU hardware: the real-backend GPU test
# (tests/test_multi_gpu_capture_gpu.py) covers the one-device case only.
_MULTI_GPU_CAPTURE = os.environ.get("LJS_MULTI_GPU_CAPTURE", "0") == "1"


_SEEDS: Dict[Tuple, torch.Tensor] = {}


# debugging switch: back-propagate a sharded scalar sum through its all-reduce (the generic
# transpose) instead of seeding the pre-reduction partial sums
_SEED_THROUGH_ALLREDUCE = os.environ.get("LJS_SEED_THROUGH_ALLREDUCE", "0") == "1"


def _seed(t: torch.Tensor, value: float) -> torch.Tensor:
    """Constant cotangent seed, cached per (device, dtype, shape, value): autograd only reads
    it, so a captured train step replays without a fill kernel."""
    key = (t.device, t.dtype, tuple(t.shape), value)
    s = _SEEDS.get(key)
    if s is None:
        s = torch.full(t.shape, value, dtype=t.dtype, device=t.device)
        if t.device.type == "meta" or (t.is_cuda and torch.cuda.is_current_stream_capturing()):
            return s
        _SEEDS[key] = s
        if t.is_cuda and t.dtype == torch.float32 and s.numel() == 1:
            # its bf16 rounding, for a bf16 sum's backward fed by this f32 seed (no cast kernel)
            from ..ops import hip as _hip
            _hip.register_seed_bf16(s, s.to(torch.bfloat16), value)
        elif t.is_cuda and t.dtype == torch.bfloat16 and s.numel() == 1:
            from ..ops import hip as _hip
            _hip.register_seed_const(s, value)
    return s


_SEED_HOIST = os.environ.get("LJS_SEED_HOIST", "1") == "1"
_REPLAY_TRACE = os.environ.get("LJS_REPLAY_TRACE", "0") == "1"


def _edge_node(t):
    """The autograd node a seed target feeds: a tensor's grad_fn, or a GradientEdge's node."""
    return t.grad_fn if isinstance(t, torch.Tensor) else t.node


def _edge_nr(t):
    # (a tensor and a GradientEdge both name their output slot output_nr)
    return t.output_nr


def _through_permutations(ts: List[torch.Tensor]):
    """The targets to seed with a summed loss's constant cotangent, as ``(target, shape, dtype,
    device)``: when ``ts`` are ALL the outputs of one all-to-all (a permutation of elements over the
    devices - e.g. the reference's final ``("batch", "length", "embed")`` constraint on the block
    output), the all-to-all's inputs instead - their gradient edges, the node keeps only their
    metadata - repeatedly.  The sum is the same either way, and the backward then runs no
    transposed all-to-all on a materialised constant (a copy, a pack and a column-sum kernel per
    step)."""
    from torch.autograd.graph import GradientEdge
    tgt = [(t, tuple(t.shape), t.dtype, t.device) for t in ts]
    if not _SEED_HOIST:
        return tgt
    while tgt:
        fn = _edge_node(tgt[0][0])
        if fn is None or type(fn).__name__ != "_CollectiveFnBackward" or getattr(fn, "perm_inputs", None) is None:
            return tgt
        meta = fn.perm_inputs
        if len(tgt) != len(meta) or any(_edge_node(t) is not fn for t, *_ in tgt) or \
                sorted(_edge_nr(t) for t, *_ in tgt) != list(range(len(meta))):
            return tgt
        edges = fn.next_functions
        if not all(m[3] for m in meta) or len(edges) != len(meta) or any(e[0] is None for e in edges):
            return tgt
        tgt = [(GradientEdge(e[0], e[1]), m[0], m[1], m[2]) for e, m in zip(edges, meta)]
        HOIST_STATS["hoisted"] += 1
    return tgt


HOIST_STATS = {"hoisted": 0}


def value_and_grad(fun: Callable, argnums=0, has_aux: bool = False):
    multi = isinstance(argnums, (tuple, list))
    argnums_t = tuple(argnums) if multi else (argnums,)

    def vg(*args, **kwargs):
        args = list(args)
        diff_leaves: List[List[ShardedArray]] = []
        for a in argnums_t:
            new = T.tree_map(lambda x: _fresh_leaf(x) if isinstance(x, ShardedArray) else x, args[a],
                             is_leaf=_leaf_is_array)
            args[a] = new
            diff_leaves.append([l for l in T.tree_leaves(new, is_leaf=_leaf_is_array) if isinstance(l, ShardedArray)])
        with torch.enable_grad():
            res = fun(*args, **kwargs)
        out, aux = (res if has_aux else (res, None))
        if not isinstance(out, ShardedArray) or out.size != 1:
            raise TypeError("grad requires a scalar-output function")
        ta = out.tile
        n_holders = ta.num_devices
        outs, seeds = [], []
        partials = getattr(out, "_sum_partials", None)
        sum_inputs = getattr(out, "_sum_inputs", None)
        if sum_inputs is not None and isinstance(out.local, LazyLocal) and out.local.pending \
                and not _SEED_THROUGH_ALLREDUCE:
            # out = sum(x) whose value nobody has read: seed x with the broadcast cotangent
            # (gsize / n_holders in x's dtype, all strides 0 - what the sum's backward returns)
            xs, gsize = sum_inputs
            for t, shape, dt, dev in _through_permutations([t for t in xs.values()]):
                outs.append(t)
                seeds.append(_seed(torch.empty((), dtype=dt, device=dev), gsize / n_holders).expand(shape))
        elif partials is not None and not _SEED_THROUGH_ALLREDUCE:
            # out = all_reduce(partials) over groups of size G (replicated over n_holders / G
            # groups): seeding each partial with G / n_holders is exactly what the all-reduce's
            # transpose would deliver to it from the 1 / n_holders seeds below
            loc, gsize = partials
            for d, t in loc.items():
                if t.requires_grad:
                    outs.append(t)
                    seeds.append(_seed(t, gsize / n_holders))
        else:
            for d, t in out.local.items():
                if t.requires_grad:
                    outs.append(t)
                    seeds.append(_seed(t, 1.0 / n_holders))
        grads_per_arg = []
        all_leaves = [l for ls in diff_leaves for l in ls]
        inputs = [t for l in all_leaves for t in l.local.values() if t.requires_grad]
        # one process per GPU: replica-group gradient sums are bucketed and overlapped with
        # the rest of the backward pass (parallel/data.py)
        from ..parallel.data import GradReducer
        reducer = None
        hooks = []
        if inputs and GradReducer.wanted(all_leaves) and all(
                len(l.local) == 1 and next(iter(l.local.values())).requires_grad for l in all_leaves):
            reducer = GradReducer(all_leaves)
            hooks = reducer.attach([next(iter(l.local.values())) for l in all_leaves])
        from . import graphs as _graphs
        try:
            if outs and inputs:
                # under a segmented capture the backward must run on this thread: HIP ends a
                # graph capture only on the thread that began it, and collectives cut captures
                from ..ops import linear as _lin
                side = reducer is None and all(t.is_cuda for t in inputs)
                # one device, no gradient all-reduce: weight-gradient combines may be left to the
                # fused Adam (ops/linear.defer_wgrads)
                one_dev = side and all(len(l.local) == 1 for l in all_leaves) and len(
                    {d for l in all_leaves for d in l.local}) == 1 and not _multi_process()
                dfr = _lin.defer_wgrads(outs, one_dev, proxies=side and not _multi_process())
                # (LJS_ATEN_TRACE: on this thread, so the tracer sees the backward's call sites)
                mt = _graphs.current() is None and not os.environ.get("LJS_ATEN_TRACE")
                with torch.autograd.set_multithreading_enabled(mt), dfr:
                    gs = torch.autograd.grad(outs, inputs, seeds, allow_unused=True)
            else:
                gs = [None] * len(inputs)
                dfr = None
        finally:
            for h in hooks:
                h.remove()
        gmap = {id(t): g for t, g in zip(inputs, gs)}
        pairs = []
        deferred = {}
        for i, l in enumerate(all_leaves):
            loc = {}
            for d, t in l.local.items():
                g = gmap.get(id(t))
                loc[d] = torch.zeros_like(t) if g is None else g
                ent = dfr.take(g) if (dfr is not None and g is not None) else None
                if ent is not None:
                    deferred[i] = (d, g, ent)
            pairs.append((l, loc))
        if dfr is not None:
            dfr.flush()
        if reducer is not None:
            red = reducer.finish({i: loc for i, (_, loc) in enumerate(pairs)})
            reduced = [red[i] for i in range(len(pairs))]
        else:
            reduced = reduce_replica_grads(pairs)
        gi = 0
        for a, ls in zip(argnums_t, diff_leaves):
            it = iter(range(gi, gi + len(ls)))
            gi += len(ls)

            def mk(x):
                if isinstance(x, ShardedArray):
                    i = next(it)
                    p = all_leaves[i]
                    r = reduced[i]
                    dfe = deferred.get(i)
                    if dfe is not None and not isinstance(r, LazyLocal) and len(r) == 1 \
                            and r.get(dfe[0]) is dfe[1]:
                        # an uncombined weight gradient: the fused Adam sums its slabs (.slabs);
                        # any other read combines it first
                        d0, g0, (desc, mat) = dfe
                        loc = LazyLocal(lambda d0=d0, g0=g0, mat=mat: (mat(), {d0: g0.detach()})[1])
                        loc.slabs = {d0: desc}
                        loc.materialize = mat
                        return ShardedArray(p.shape, p.dtype, p.sharding, loc)
                    if dfe is not None:
                        # taken out of the deferral but not handed over as slabs: combine it now
                        # (flush() no longer sees it)
                        dfe[2][1]()
                    if isinstance(r, LazyLocal) and r.pending:
                        # keep a reduced-in-wire-dtype gradient lazy (the optimizer reads .raw)
                        loc = LazyLocal(lambda r=r: {d: t.detach() for d, t in r.items()})
                        loc.raw = {d: t.detach() for d, t in r.raw.items()}
                    else:
                        loc = {d: t.detach() for d, t in r.items()}
                    return ShardedArray(p.shape, p.dtype, p.sharding, loc)
                return x
            grads_per_arg.append(T.tree_map(mk, args[a], is_leaf=_leaf_is_array))
        g = tuple(grads_per_arg) if multi else grads_per_arg[0]
        if isinstance(out.local, LazyLocal) and out.local.pending:
            # the value of a lazily all-reduced scalar stays lazy: grad() drops it unread
            val = ShardedArray(out.shape, out.dtype, out.sharding,
                               LazyLocal(lambda o=out: {d: t.detach() for d, t in o.local.items()}))
        else:
            val = ShardedArray(out.shape, out.dtype, out.sharding, {d: t.detach() for d, t in out.local.items()})
        if has_aux:
            return (val, aux), g
        return val, g

    return vg


def grad(fun: Callable, argnums=0, has_aux: bool = False):
    vg = value_and_grad(fun, argnums, has_aux)

    def g_clean(*args, **kwargs):
        if has_aux:
            (val, aux), grads = vg(*args, **kwargs)
            return grads, aux
        return vg(*args, **kwargs)[1]

    return g_clean


# ----------------------------------------------------------------------------- eval_shape
def _to_abstract(x):
    if isinstance(x, ShardedArray):
        loc = {d: torch.empty(t.shape, dtype=t.dtype, device="meta") for d, t in x.local.items()}
        return ShardedArray(x.shape, x.dtype, x.sharding, loc)
    if isinstance(x, ShapeDtypeStruct):
        from ..runtime.devices import devices
        sh = x.sharding or SingleDeviceSharding(devices()[0])
        ta = sh.tile_assignment(len(x.shape))
        loc = {d: torch.empty(ta.shard_shape(x.shape), dtype=x.dtype, device="meta") for d in ta.device_ids
               if _addressable(d)}
        return ShardedArray(x.shape, x.dtype, sh, loc)
    return x


def _addressable(d):
    from ..runtime.devices import get_device, process_index
    return get_device(d).process_index == process_index()


def eval_shape(fun: Callable, *args, **kwargs):
    a2 = T.tree_map(_to_abstract, list(args), is_leaf=lambda x: isinstance(x, (ShardedArray, ShapeDtypeStruct)))
    with _state.abstract(), torch.no_grad():
        out = fun(*a2, **kwargs)
    return T.tree_map(lambda x: ShapeDtypeStruct(x.shape, x.dtype) if isinstance(x, ShardedArray) else x, out,
                      is_leaf=_leaf_is_array)
