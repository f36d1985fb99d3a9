"""``flax.linen.Module`` equivalent: dataclass modules with ``setup`` / ``@compact``.

Reference usage: ``class FlaxAttention(nn.Module)`` with dataclass fields and
``setup()`` (``case6_attention.py:42-91``) or ``@nn.compact`` (``case5_attention_dense.py:52-71``);
``model.init(rngs, x)`` -> ``{'params': ...}`` (``case6_attention.py:172``);
``model.apply({'params': p}, x)`` (``case6_attention.py:210``).

Parameters are :class:`ShardedArray` leaves in a nested dict, optionally boxed
in :class:`~.partitioning.Partitioned` with logical axis names.  A parameter's
random stream is derived from its path, so initialisation is deterministic and
independent of the order modules are built in.
"""
from __future__ import annotations

import copy
import dataclasses
import functools
import threading
import zlib
from typing import Any, Callable, Dict, Optional, Tuple

from .. import random as _random
from ..utils import tree as T
from .partitioning import Partitioned

__all__ = ["Module", "compact", "Scope"]

_TLS = threading.local()


def _ctx_stack():
    s = getattr(_TLS, "stack", None)
    if s is None:
        s = _TLS.stack = []
    return s


class Scope:
    def __init__(self, params: Dict[str, Any], rngs: Dict[str, Any], mode: str, path: Tuple[str, ...] = ()):
        self.params = params
        self.rngs = rngs
        self.mode = mode
        self.path = path

    def child(self, name: str) -> "Scope":
        sub = self.params.get(name)
        if sub is None:
            if self.mode != "init":
                sub = {}
            else:
                sub = self.params.setdefault(name, {})
        return Scope(sub, self.rngs, self.mode, self.path + (name,))

    def make_rng(self, kind: str, salt: str = ""):
        k = self.rngs.get(kind)
        if k is None:
            raise ValueError(f"no PRNG key for stream {kind!r} (pass rngs={{'{kind}': key}})")
        h = zlib.crc32(("/".join(self.path) + "#" + salt).encode())
        return _random.fold_in(k, h)


def _prune(d: Dict[str, Any]) -> Dict[str, Any]:
    """Drop sub-module entries that created no parameters (flax omits them)."""
    out = {}
    for k, v in d.items():
        if isinstance(v, dict):
            v = _prune(v)
            if not v:
                continue
        out[k] = v
    return out


def compact(fn: Callable) -> Callable:
    fn._ljs_compact = True
    return fn


def _wrap_method(fn: Callable, kind: str) -> Callable:
    @functools.wraps(fn)
    def wrapped(self, *args, **kwargs):
        if getattr(self, "_scope", None) is None:
            return fn(self, *args, **kwargs)
        self._ensure_setup()
        st = _ctx_stack()
        st.append((kind, self))
        object.__setattr__(self, "_autoname", {})
        try:
            return fn(self, *args, **kwargs)
        finally:
            st.pop()
    wrapped._ljs_wrapped = True
    return wrapped


@dataclasses.dataclass(eq=False, repr=False)
class Module:
    name: Optional[str] = dataclasses.field(default=None, kw_only=True)

    def __init_subclass__(cls, **kwargs):
        super().__init_subclass__(**kwargs)
        dataclasses.dataclass(cls, eq=False, repr=False)
        for attr in list(vars(cls)):
            fn = vars(cls)[attr]
            if not callable(fn) or getattr(fn, "_ljs_wrapped", False) or isinstance(fn, (staticmethod, classmethod)):
                continue
            if attr == "__call__" or getattr(fn, "_ljs_compact", False):
                setattr(cls, attr, _wrap_method(fn, "compact" if getattr(fn, "_ljs_compact", False) else "call"))

    def __post_init__(self):
        object.__setattr__(self, "_scope", None)
        object.__setattr__(self, "_setup_done", False)
        object.__setattr__(self, "_autoname", {})
        st = _ctx_stack()
        if st:
            kind, parent = st[-1]
            if kind == "compact" and parent._scope is not None:
                n = self.name
                if n is None:
                    cnt = parent._autoname.get(type(self).__name__, 0)
                    parent._autoname[type(self).__name__] = cnt + 1
                    n = f"{type(self).__name__}_{cnt}"
                self._bind_inplace(parent._scope.child(n), n)

    # ------------------------------------------------------------------ binding
    def _bind_inplace(self, scope: Scope, name: Optional[str] = None):
        object.__setattr__(self, "_scope", scope)
        if name is not None and self.name is None:
            object.__setattr__(self, "name", name)
        object.__setattr__(self, "_setup_done", False)

    def _ensure_setup(self):
        if not self._setup_done and self._scope is not None:
            object.__setattr__(self, "_setup_done", True)
            st = _ctx_stack()
            st.append(("setup", self))
            try:
                self.setup()
            finally:
                st.pop()

    def __setattr__(self, key, value):
        scope = self.__dict__.get("_scope")
        if scope is not None and not key.startswith("_"):
            value = self._register_children(key, value)
        object.__setattr__(self, key, value)

    def _register_children(self, key, value):
        scope = self._scope
        if isinstance(value, Module):
            if value._scope is None:
                n = value.name or key
                value._bind_inplace(scope.child(n), n)
            return value
        if isinstance(value, (list, tuple)) and any(isinstance(v, Module) for v in value):
            out = []
            for i, v in enumerate(value):
                if isinstance(v, Module) and v._scope is None:
                    n = v.name or f"{key}_{i}"
                    v._bind_inplace(scope.child(n), n)
                out.append(v)
            return type(value)(out)
        return value

    def __getattr__(self, item):
        # attributes created in setup(): run setup lazily on first access
        d = self.__dict__
        if not item.startswith("_") and d.get("_scope") is not None and not d.get("_setup_done"):
            self._ensure_setup()
            if item in self.__dict__:
                return self.__dict__[item]
        raise AttributeError(f"{type(self).__name__!r} object has no attribute {item!r}")

    def setup(self):
        pass

    # ------------------------------------------------------------------ params / rngs
    @property
    def scope(self) -> Scope:
        if self._scope is None:
            raise RuntimeError("unbound module: call it through .init / .apply")
        return self._scope

    def param(self, name: str, init_fn: Callable, *init_args, unbox: bool = True):
        scope = self.scope
        if name in scope.params:
            v = scope.params[name]
        elif scope.mode == "init":
            v = init_fn(scope.make_rng("params", name), *init_args)
            scope.params[name] = v
        else:
            raise KeyError(f"parameter {'/'.join(scope.path + (name,))} not found in variables")
        if unbox and isinstance(v, Partitioned):
            return v.value
        return v

    def make_rng(self, kind: str = "params"):
        return self.scope.make_rng(kind)

    @property
    def is_initializing(self) -> bool:
        return self._scope is not None and self._scope.mode == "init"

    # ------------------------------------------------------------------ entry points
    def _clone_bound(self, scope: Scope) -> "Module":
        m = copy.copy(self)
        object.__setattr__(m, "_scope", scope)
        object.__setattr__(m, "_setup_done", False)
        object.__setattr__(m, "_autoname", {})
        return m

    @staticmethod
    def _rngs(rngs):
        if rngs is None:
            return {}
        if isinstance(rngs, dict):
            return dict(rngs)
        return {"params": rngs}

    def init(self, rngs, *args, method=None, **kwargs) -> Dict[str, Any]:
        params: Dict[str, Any] = {}
        m = self._clone_bound(Scope(params, self._rngs(rngs), "init"))
        fn = getattr(m, method) if isinstance(method, str) else (method.__get__(m) if method else m)
        fn(*args, **kwargs)
        return {"params": _prune(params)}

    def init_with_output(self, rngs, *args, method=None, **kwargs):
        params: Dict[str, Any] = {}
        m = self._clone_bound(Scope(params, self._rngs(rngs), "init"))
        fn = getattr(m, method) if isinstance(method, str) else (method.__get__(m) if method else m)
        out = fn(*args, **kwargs)
        return out, {"params": _prune(params)}

    def apply(self, variables, *args, rngs=None, method=None, mutable=False, **kwargs):
        params = variables.get("params", {}) if isinstance(variables, dict) else variables
        m = self._clone_bound(Scope(params, self._rngs(rngs), "apply"))
        fn = getattr(m, method) if isinstance(method, str) else (method.__get__(m) if method else m)
        out = fn(*args, **kwargs)
        if mutable:
            return out, {}
        return out

    def __repr__(self):
        fields = ", ".join(f"{f.name}={getattr(self, f.name)!r}" for f in dataclasses.fields(self)
                           if f.name != "name")
        return f"{type(self).__name__}({fields})"
