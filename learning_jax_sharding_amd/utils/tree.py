"""Minimal pytree utilities (``jax.tree_util`` subset).

Containers: dict (sorted keys, like JAX), list, tuple, namedtuple, None (empty),
plus classes registered with :func:`register_pytree_node` (TrainState, the
``Partitioned`` box of ``nn``).
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Tuple

__all__ = [
    "register_pytree_node",
    "tree_flatten",
    "tree_unflatten",
    "tree_map",
    "tree_leaves",
    "tree_structure",
    "is_container",
    "TreeDef",
]

_REGISTRY: Dict[type, Tuple[Callable, Callable]] = {}


def register_pytree_node(cls, flatten: Callable, unflatten: Callable) -> None:
    """``flatten(x) -> (children, aux)``; ``unflatten(aux, children) -> x``."""
    _REGISTRY[cls] = (flatten, unflatten)


def _is_namedtuple(x) -> bool:
    return isinstance(x, tuple) and hasattr(x, "_fields")


def is_container(x) -> bool:
    if getattr(type(x), "__pytree_leaf__", False):
        return False
    return (x is None or isinstance(x, (dict, list, tuple)) or type(x) in _REGISTRY)


class TreeDef:
    __slots__ = ("kind", "aux", "children", "num_leaves")

    def __init__(self, kind, aux, children):
        self.kind = kind
        self.aux = aux
        self.children = children
        self.num_leaves = 1 if kind == "leaf" else sum(c.num_leaves for c in children)

    def __eq__(self, other):
        return (isinstance(other, TreeDef) and self.kind == other.kind and self.aux == other.aux
                and self.children == other.children)

    def __hash__(self):
        return hash((self.kind if not isinstance(self.kind, type) else self.kind.__name__,
                     _hashable(self.aux), tuple(self.children)))

    def __repr__(self):
        if self.kind == "leaf":
            return "*"
        return f"{getattr(self.kind, '__name__', self.kind)}({self.aux!r}, {self.children})"


def _hashable(x):
    try:
        hash(x)
        return x
    except TypeError:
        return repr(x)


def _flatten(x, leaves: List[Any], is_leaf) -> TreeDef:
    if is_leaf is not None and is_leaf(x):
        leaves.append(x)
        return TreeDef("leaf", None, [])
    if x is None:
        return TreeDef("none", None, [])
    t = type(x)
    if getattr(t, "__pytree_leaf__", False):
        leaves.append(x)
        return TreeDef("leaf", None, [])
    if t in _REGISTRY:
        children, aux = _REGISTRY[t][0](x)
        return TreeDef(t, aux, [_flatten(c, leaves, is_leaf) for c in children])
    if isinstance(x, dict):
        keys = sorted(x.keys(), key=lambda k: (str(type(k)), k))
        return TreeDef(type(x) if type(x) is not dict else "dict", tuple(keys),
                       [_flatten(x[k], leaves, is_leaf) for k in keys])
    if _is_namedtuple(x):
        return TreeDef(type(x), None, [_flatten(c, leaves, is_leaf) for c in x])
    if isinstance(x, tuple):
        return TreeDef("tuple", len(x), [_flatten(c, leaves, is_leaf) for c in x])
    if isinstance(x, list):
        return TreeDef("list", len(x), [_flatten(c, leaves, is_leaf) for c in x])
    leaves.append(x)
    return TreeDef("leaf", None, [])


def tree_flatten(tree, is_leaf=None):
    leaves: List[Any] = []
    td = _flatten(tree, leaves, is_leaf)
    return leaves, td


def tree_leaves_with_path(tree, is_leaf=None) -> List[Tuple[Tuple[Any, ...], Any]]:
    """``[(path, leaf)]`` in :func:`tree_flatten` order; path entries are dict keys, sequence
    indices, namedtuple field names or child indices of registered nodes."""
    out: List[Tuple[Tuple[Any, ...], Any]] = []

    def walk(x, path):
        if is_leaf is not None and is_leaf(x):
            out.append((path, x))
            return
        if x is None:
            return
        t = type(x)
        if getattr(t, "__pytree_leaf__", False):
            out.append((path, x))
        elif t in _REGISTRY:
            children, _ = _REGISTRY[t][0](x)
            names = getattr(x, "__pytree_child_names__", None)
            for i, c in enumerate(children):
                walk(c, path + ((names[i] if names else i),))
        elif isinstance(x, dict):
            for k in sorted(x.keys(), key=lambda k: (str(type(k)), k)):
                walk(x[k], path + (k,))
        elif _is_namedtuple(x):
            for f, c in zip(x._fields, x):
                walk(c, path + (f,))
        elif isinstance(x, (tuple, list)):
            for i, c in enumerate(x):
                walk(c, path + (i,))
        else:
            out.append((path, x))

    walk(tree, ())
    return out


def _unflatten(td: TreeDef, it):
    k = td.kind
    if k == "leaf":
        return next(it)
    if k == "none":
        return None
    kids = [_unflatten(c, it) for c in td.children]
    if k == "dict":
        return dict(zip(td.aux, kids))
    if k == "tuple":
        return tuple(kids)
    if k == "list":
        return list(kids)
    if isinstance(k, type) and k in _REGISTRY:
        return _REGISTRY[k][1](td.aux, kids)
    if isinstance(k, type) and issubclass(k, dict):
        return k(zip(td.aux, kids))
    if isinstance(k, type) and issubclass(k, tuple):
        return k(*kids)
    raise TypeError(f"cannot unflatten node kind {k}")


def tree_unflatten(td: TreeDef, leaves):
    it = iter(leaves)
    out = _unflatten(td, it)
    return out


def tree_leaves(tree, is_leaf=None):
    return tree_flatten(tree, is_leaf)[0]


def tree_structure(tree, is_leaf=None):
    return tree_flatten(tree, is_leaf)[1]


def tree_map(f, tree, *rest, is_leaf=None):
    leaves, td = tree_flatten(tree, is_leaf)
    # extra trees may be prefixes of ``tree`` (a leaf, incl. None, covers a whole subtree)
    others = [_broadcast_prefix(r, tree, is_leaf) for r in rest]
    return tree_unflatten(td, [f(x, *[o[i] for o in others]) for i, x in enumerate(leaves)])


def broadcast_prefix(prefix, full, is_leaf=None):
    return _broadcast_prefix(prefix, full, is_leaf)


def _broadcast_prefix(prefix, full, is_leaf):
    """Expand a prefix tree so each of its leaves covers the matching subtree of ``full``."""
    out: List[Any] = []

    def rec(p, f):
        if is_container(f) and not (is_leaf and is_leaf(f)) and is_container(p) and p is not None:
            pl, ptd = tree_flatten(p, is_leaf=lambda x: x is not p)
            fl, ftd = tree_flatten(f, is_leaf=lambda x: x is not f)
            if ptd.kind != ftd.kind or len(pl) != len(fl) or (ptd.kind == "dict" and ptd.aux != ftd.aux):
                raise ValueError(f"tree prefix does not match: {ptd} vs {ftd}")
            for a, b in zip(pl, fl):
                rec(a, b)
        else:
            n = len(tree_leaves(f, is_leaf))
            out.extend([p] * n)

    rec(prefix, full)
    return out
