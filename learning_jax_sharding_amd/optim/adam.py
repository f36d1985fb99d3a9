"""Optimizers (``optax`` subset): Adam/AdamW/SGD with a fused MI355X update.

Reference usage: ``optax.adam(learning_rate=0.001)`` (``case6_attention.py:181``)
and ``state.apply_gradients(grads=grads)`` (``case6_attention.py:214``).
State layout mirrors optax - ``(ScaleByAdamState(count, mu, nu), EmptyState())``
- so ``mu``/``nu`` inherit the parameter shardings through the logical boxes
and ``get_partition_spec`` shards them like the params.

The update itself is one fused HIP kernel per local shard (``ljs_adam_f32``):
``m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= lr_t m / (sqrt(v) + eps_t)``
with the bias correction computed on device from the step counter, so the
whole update is HIP-graph capturable.  Inside a ``jit(..., donate_argnums=0)``
the update is in place (no new parameter buffers).
"""
from __future__ import annotations

from typing import Any, Callable, NamedTuple, Optional

import torch

from ..array import ShardedArray
from ..ops import optim_kernels as OK
from ..spmd import state as _state
from ..utils import tree as T

__all__ = ["GradientTransformation", "ScaleByAdamState", "EmptyState", "adam", "adamw", "sgd", "apply_updates",
           "chain", "scale"]


class EmptyState(NamedTuple):
    pass


class ScaleByAdamState(NamedTuple):
    count: Any
    mu: Any
    nu: Any


class GradientTransformation(NamedTuple):
    init: Callable
    update: Callable


def _is_arr(x):
    return isinstance(x, ShardedArray)


def _zeros_like(x: ShardedArray) -> ShardedArray:
    return ShardedArray(x.shape, x.dtype, x.sharding, {d: torch.zeros_like(t) for d, t in x.local.items()})


def _counter_like(params) -> ShardedArray:
    """int32 scalar step counter, replicated on the params' devices."""
    leaves = [l for l in T.tree_leaves(params, is_leaf=_is_arr) if _is_arr(l)]
    from ..sharding.shardings import GSPMDSharding
    from ..sharding.tile import TileAssignment
    if not leaves:
        from ..array import device_put
        return device_put(torch.zeros((), dtype=torch.int32))
    p0 = leaves[0]
    devs = sorted(set(d for l in leaves for d in l.tile.device_ids))
    sh = GSPMDSharding(tuple(p0.sharding._device_assignment), TileAssignment.replicated(devs, 0))
    loc = {}
    for l in leaves:
        for d, t in l.local.items():
            if d not in loc:
                loc[d] = torch.zeros((), dtype=torch.int32, device=t.device)
    return ShardedArray((), torch.int32, sh, loc)


def apply_updates(params, updates):
    def add(p, u):
        if not _is_arr(p):
            return p
        return ShardedArray(p.shape, p.dtype, p.sharding,
                            {d: (t + u.local[d].to(t.dtype)) for d, t in p.local.items()})
    return T.tree_map(add, params, updates, is_leaf=_is_arr)


class _Adam:
    """A GradientTransformation-compatible object with a fused ``apply`` fast path."""

    def __init__(self, learning_rate: float, b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8,
                 weight_decay: float = 0.0):
        self.learning_rate = learning_rate
        self.b1, self.b2, self.eps = b1, b2, eps
        self.weight_decay = weight_decay

    def __hash__(self):
        return hash(("adam", self.learning_rate, self.b1, self.b2, self.eps, self.weight_decay))

    def __eq__(self, other):
        return isinstance(other, _Adam) and hash(self) == hash(other)

    def init(self, params):
        mu = T.tree_map(lambda p: _zeros_like(p) if _is_arr(p) else p, params, is_leaf=_is_arr)
        nu = T.tree_map(lambda p: _zeros_like(p) if _is_arr(p) else p, params, is_leaf=_is_arr)
        return (ScaleByAdamState(_counter_like(params), mu, nu), EmptyState())

    def _lr(self):
        lr = self.learning_rate
        return float(lr) if not callable(lr) else lr

    def update(self, grads, state, params=None):
        """optax-style: returns (updates, new_state); updates are added with :func:`apply_updates`."""
        st, empty = state
        count = st.count
        new_count = ShardedArray((), torch.int32, count.sharding, {d: t + 1 for d, t in count.local.items()})
        upd, mus, nus = {}, {}, {}

        def one(g, m, v, p=None):
            if not _is_arr(g):
                return g, m, v
            lu, lm, lv = {}, {}, {}
            for d, gt in g.local.items():
                u, m2, v2 = OK.adam_moments_and_update(gt, m.local[d], v.local[d], new_count.local[d],
                                                       self._lr(), self.b1, self.b2, self.eps,
                                                       None if p is None else p.local[d], self.weight_decay)
                lu[d], lm[d], lv[d] = u, m2, v2
            mk = lambda loc: ShardedArray(g.shape, g.dtype, g.sharding, loc)  # noqa: E731
            return mk(lu), mk(lm), mk(lv)

        gl, gtd = T.tree_flatten(grads, is_leaf=_is_arr)
        ml = T.tree_leaves(st.mu, is_leaf=_is_arr)
        vl = T.tree_leaves(st.nu, is_leaf=_is_arr)
        pl = T.tree_leaves(params, is_leaf=_is_arr) if params is not None else [None] * len(gl)
        res = [one(g, m, v, p) for g, m, v, p in zip(gl, ml, vl, pl)]
        updates = T.tree_unflatten(gtd, [r[0] for r in res])
        mu = T.tree_unflatten(T.tree_structure(st.mu, is_leaf=_is_arr), [r[1] for r in res])
        nu = T.tree_unflatten(T.tree_structure(st.nu, is_leaf=_is_arr), [r[2] for r in res])
        return updates, (ScaleByAdamState(new_count, mu, nu), empty)

    def apply(self, params, grads, state):
        """Fused ``update`` + ``apply_updates``: one kernel per shard; in place when donated."""
        st, empty = state
        count = st.count
        inplace = all(_state.is_donated(t) for t in dict.values(count.local))
        pl, ptd = T.tree_flatten(params, is_leaf=_is_arr)
        gl = T.tree_leaves(grads, is_leaf=_is_arr)
        ml = T.tree_leaves(st.mu, is_leaf=_is_arr)
        vl = T.tree_leaves(st.nu, is_leaf=_is_arr)
        # multi-tensor kernel; with a donated counter it also performs the count increment
        fused = self._apply_multi(pl, gl, ml, vl, count, inplace)
        if fused is not None:
            new_p, new_m, new_v, new_count = fused
            params2 = T.tree_unflatten(ptd, new_p)
            mu = T.tree_unflatten(T.tree_structure(st.mu, is_leaf=_is_arr), new_m)
            nu = T.tree_unflatten(T.tree_structure(st.nu, is_leaf=_is_arr), new_v)
            return params2, (ScaleByAdamState(new_count, mu, nu), empty)
        if inplace:
            for t in count.local.values():
                t.add_(1)
            new_count = count
        else:
            new_count = ShardedArray((), torch.int32, count.sharding, {d: t + 1 for d, t in count.local.items()})
        new_p, new_m, new_v = [], [], []
        for p, g, m, v in zip(pl, gl, ml, vl):
            if not _is_arr(p):
                new_p.append(p), new_m.append(m), new_v.append(v)
                continue
            lp, lm, lv = {}, {}, {}
            for d, pt in p.local.items():
                ip = inplace and _state.is_donated(pt)
                lp[d], lm[d], lv[d] = OK.adam_fused(pt, g.local[d], m.local[d], v.local[d], new_count.local[d],
                                                    self._lr(), self.b1, self.b2, self.eps, self.weight_decay,
                                                    inplace=ip)
            new_p.append(ShardedArray(p.shape, p.dtype, p.sharding, lp))
            new_m.append(ShardedArray(m.shape, m.dtype, m.sharding, lm))
            new_v.append(ShardedArray(v.shape, v.dtype, v.sharding, lv))
        params2 = T.tree_unflatten(ptd, new_p)
        mu = T.tree_unflatten(T.tree_structure(st.mu, is_leaf=_is_arr), new_m)
        nu = T.tree_unflatten(T.tree_structure(st.nu, is_leaf=_is_arr), new_v)
        return params2, (ScaleByAdamState(new_count, mu, nu), empty)


def _grad_local(g: ShardedArray, d: int) -> torch.Tensor:
    """Gradient shard for the fused kernel: a data-parallel gradient still in its bf16 wire
    buffer is read there (the kernel converts on load) instead of being cast back to f32."""
    loc = g.local
    slabs = getattr(loc, "slabs", None)
    if slabs is not None and getattr(loc, "pending", False) and d in slabs:
        return slabs[d]  # hip.SlabGrad / hip.ConstGrad: summed (or broadcast) inside the kernel
    raw = getattr(loc, "raw", None)
    if raw is not None and getattr(loc, "pending", False) and d in raw:
        return raw[d]
    return loc[d]


class CountLocal(dict):
    """Local tensors of a step counter whose increments may be deferred inside a multi-step
    graph capture (ops/hip._defer_step_inc: one count launch per graph).  The next Adam launch
    adds the pending offset itself and reads the dict raw (``dict.items``); any OTHER read from a
    jitted function's body -- ``state.step`` folded into an RNG key, an LR schedule -- first
    launches the pending increments, so in-graph reads see the same count as eager steps."""

    def _flush(self):
        if _state.in_user_code():
            from ..ops import hip
            for t in dict.values(self):
                hip.flush_step_inc(t)
        return self

    def __getitem__(self, k):
        return dict.__getitem__(self._flush(), k)

    def __iter__(self):
        return dict.__iter__(self._flush())

    def values(self):
        return dict.values(self._flush())

    def items(self):
        return dict.items(self._flush())

    def get(self, k, default=None):
        return dict.get(self._flush(), k, default)


def _raw(count: ShardedArray) -> dict:
    return dict(dict.items(count.local))


def _adam_multi_apply(self, pl, gl, ml, vl, count, inplace):
    """MI355X path: every local shard of every param in ONE multi-tensor kernel per device
    (it also refreshes the params' bf16 GEMM shadows).  Returns None to use the per-leaf path."""
    arrs = [(p, g, m, v) for p, g, m, v in zip(pl, gl, ml, vl) if _is_arr(p)]
    if not arrs or len(arrs) != len(pl):
        return None
    for p, g, m, v in arrs:
        for d, t in p.local.items():
            if not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous():
                return None
            if not (m.local[d].is_contiguous() and v.local[d].is_contiguous()):
                return None
    from ..ops import hip
    new_loc = [({}, {}, {}) for _ in arrs]
    by_dev = {}
    for i, (p, g, m, v) in enumerate(arrs):
        for d, pt in p.local.items():
            mt, vt = m.local[d], v.local[d]
            if inplace and _state.is_donated(pt):
                tp, tm, tv = pt, mt, vt
            else:
                tp, tm, tv = pt.clone(), mt.clone(), vt.clone()
            new_loc[i][0][d], new_loc[i][1][d], new_loc[i][2][d] = tp, tm, tv
            by_dev.setdefault(d, []).append((tp, _grad_local(g, d), tm, tv))
    cl = _raw(count)
    fold = inplace and all(t.dtype == torch.int32 and t.is_cuda for t in cl.values()) and set(cl) == set(by_dev)
    if fold:
        # incremented in place (one-lane launch, deferred inside a capture); reads of the returned
        # counter from the jitted body flush the deferred increments first (CountLocal)
        new_count = ShardedArray((), torch.int32, count.sharding, {})
        new_count.local = CountLocal(cl)
    else:
        new_count = ShardedArray((), torch.int32, count.sharding, {d: t + 1 for d, t in cl.items()})
    nl = _raw(new_count)
    for d, entries in by_dev.items():
        hip.adam_multi(entries, nl[d], self._lr(), self.b1, self.b2, self.eps, self.weight_decay,
                       increment_step=fold)
    mk = lambda a, loc: ShardedArray(a.shape, a.dtype, a.sharding, loc)  # noqa: E731
    return ([mk(a[0], l[0]) for a, l in zip(arrs, new_loc)], [mk(a[2], l[1]) for a, l in zip(arrs, new_loc)],
            [mk(a[3], l[2]) for a, l in zip(arrs, new_loc)], new_count)


_Adam._apply_multi = _adam_multi_apply


def adam(learning_rate: float, b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8, eps_root: float = 0.0):
    return _Adam(learning_rate, b1, b2, eps)


def adamw(learning_rate: float, b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8, weight_decay: float = 1e-4):
    return _Adam(learning_rate, b1, b2, eps, weight_decay)


def scale(step_size: float) -> GradientTransformation:
    def init(params):
        return EmptyState()

    def update(grads, state, params=None):
        return T.tree_map(lambda g: ShardedArray(g.shape, g.dtype, g.sharding,
                                                 {d: t * step_size for d, t in g.local.items()})
                          if _is_arr(g) else g, grads, is_leaf=_is_arr), state
    return GradientTransformation(init, update)


def sgd(learning_rate: float) -> GradientTransformation:
    return scale(-learning_rate)


def chain(*txs) -> GradientTransformation:
    def init(params):
        return tuple(t.init(params) for t in txs)

    def update(grads, state, params=None):
        new = []
        for t, s in zip(txs, state):
            grads, s2 = t.update(grads, s, params)
            new.append(s2)
        return grads, tuple(new)
    return GradientTransformation(init, update)
