"""Logical-axis partitioning (``flax.linen.partitioning`` equivalent).

Reference usage:
* ``nn.with_logical_partitioning(init, ('embed','heads'))`` - ``case6_attention.py:56-59``
* ``nn.get_partition_spec(tree)`` - ``case6_attention.py:190``
* ``nn.logical_to_mesh_sharding(spec, mesh, rules)`` - ``case6_attention.py:191``
* ``nn_partitioning.axis_rules(rules)`` - ``case6_attention.py:219``
* ``nn.with_logical_constraint(x, names)`` - ``case6_attention.py:105-116,137,141``
"""
from __future__ import annotations

import threading
from contextlib import contextmanager
from typing import Any, Callable, Optional, Sequence, Tuple

from ..array import ShapeDtypeStruct, ShardedArray
from ..mesh import Mesh, current_mesh
from ..sharding.shardings import NamedSharding, PartitionSpec
from ..utils import tree as T

__all__ = [
    "Partitioned", "with_logical_partitioning", "get_partition_spec", "logical_to_mesh_axes",
    "logical_to_mesh_sharding", "logical_to_mesh", "axis_rules", "get_axis_rules", "with_logical_constraint",
    "unbox", "LogicallyPartitioned",
]

_TLS = threading.local()


class Partitioned:
    """A parameter boxed with its logical axis names (``nn.Partitioned``)."""

    def __init__(self, value, names: Tuple[Optional[str], ...], mesh: Optional[Mesh] = None):
        self.value = value
        self.names = tuple(names)
        self.mesh = mesh

    def unbox(self):
        return self.value

    def replace_boxed(self, v):
        return Partitioned(v, self.names, self.mesh)

    def get_partition_spec(self) -> PartitionSpec:
        return PartitionSpec(*self.names)

    @property
    def shape(self):
        return self.value.shape

    @property
    def dtype(self):
        return self.value.dtype

    def __repr__(self):
        return f"Partitioned(value={self.value!r}, names={self.names})"


LogicallyPartitioned = Partitioned
Partitioned.__pytree_child_names__ = ("value",)

T.register_pytree_node(Partitioned, lambda p: ((p.value,), (p.names, p.mesh)),
                       lambda aux, ch: Partitioned(ch[0], aux[0], aux[1]))


def unbox(tree):
    return T.tree_map(lambda x: x.value if isinstance(x, Partitioned) else x, tree,
                      is_leaf=lambda x: isinstance(x, Partitioned))


def with_logical_partitioning(fn: Callable, names: Sequence[Optional[str]], mesh: Optional[Mesh] = None,
                              rules=None) -> Callable:
    names = tuple(names)

    def init(*args, **kwargs):
        return Partitioned(fn(*args, **kwargs), names, mesh)

    init.__wrapped__ = fn
    return init


def _is_box_or_array(x):
    return isinstance(x, (Partitioned, ShardedArray, ShapeDtypeStruct))


def get_partition_spec(tree):
    """Boxed leaves -> ``PartitionSpec(*names)``; other arrays -> ``PartitionSpec()`` (replicated)."""
    def spec(x):
        if isinstance(x, Partitioned):
            return x.get_partition_spec()
        if isinstance(x, (ShardedArray, ShapeDtypeStruct)):
            return PartitionSpec()
        return None
    return T.tree_map(spec, tree, is_leaf=_is_box_or_array)


@contextmanager
def axis_rules(rules):
    prev = getattr(_TLS, "rules", None)
    _TLS.rules = tuple(tuple(r) for r in rules)
    try:
        yield
    finally:
        _TLS.rules = prev


def get_axis_rules():
    return getattr(_TLS, "rules", None) or ()


def logical_to_mesh_axes(names: Sequence[Optional[str]], rules=None) -> PartitionSpec:
    """Map logical names to mesh axes (flax's algorithm).

    Rules are walked in order; a rule ``(logical, mesh_axis)`` assigns
    ``mesh_axis`` to the first dim named ``logical`` if that dim is still
    unassigned and ``mesh_axis`` is not yet used by this array.  Unmatched
    names become ``None`` (replicated).
    """
    if rules is None:
        rules = get_axis_rules()
    names = tuple(names)
    result: list = [_UNASSIGNED] * len(names)
    for logical, mesh_axes in rules:
        if logical in names:
            pos = names.index(logical)
            axes = mesh_axes if isinstance(mesh_axes, (tuple, list)) else (mesh_axes,)
            used = set()
            for r in result:
                if r is _UNASSIGNED or r is None:
                    continue
                used.update(r if isinstance(r, tuple) else (r,))
            if result[pos] is _UNASSIGNED and not (set(a for a in axes if a is not None) & used):
                result[pos] = mesh_axes if not isinstance(mesh_axes, list) else tuple(mesh_axes)
    return PartitionSpec(*[None if r is _UNASSIGNED else r for r in result])


class _Unassigned:
    def __repr__(self):
        return "UNASSIGNED"


_UNASSIGNED = _Unassigned()


def logical_to_mesh(tree, rules=None):
    return T.tree_map(lambda s: logical_to_mesh_axes(s, rules) if isinstance(s, PartitionSpec) else s, tree,
                      is_leaf=lambda x: isinstance(x, PartitionSpec))


def logical_to_mesh_sharding(tree, mesh: Mesh, rules=None):
    def conv(s):
        if isinstance(s, PartitionSpec):
            return NamedSharding(mesh, logical_to_mesh_axes(s, rules))
        return s
    return T.tree_map(conv, tree, is_leaf=lambda x: isinstance(x, PartitionSpec))


def with_logical_constraint(x, logical_axis_resources, mesh: Optional[Mesh] = None, rules=None):
    """Reshard ``x`` to the mesh sharding of its logical names; a no-op with no mesh/rules in context."""
    mesh = mesh or current_mesh()
    rules = rules if rules is not None else get_axis_rules()
    if mesh is None or not rules:
        return x
    from ..ops.core import with_sharding_constraint
    spec = logical_to_mesh_axes(tuple(logical_axis_resources), rules)
    if isinstance(x, Partitioned):
        return x.replace_boxed(with_sharding_constraint(x.value, NamedSharding(mesh, spec)))
    return with_sharding_constraint(x, NamedSharding(mesh, spec))
