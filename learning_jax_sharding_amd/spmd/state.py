"""Thread-local execution state shared by the spmd front-ends."""
from __future__ import annotations

import threading
from contextlib import contextmanager

_TLS = threading.local()


def abstract_mode() -> bool:
    return getattr(_TLS, "abstract", 0) > 0


@contextmanager
def abstract():
    _TLS.abstract = getattr(_TLS, "abstract", 0) + 1
    try:
        yield
    finally:
        _TLS.abstract -= 1


def default_placement():
    s = getattr(_TLS, "placement", None)
    return s[-1] if s else None


@contextmanager
def placement(sharding):
    """Inside ``jit``: unplaced arrays are created replicated on the jit's devices, not device 0."""
    s = getattr(_TLS, "placement", None)
    if s is None:
        s = _TLS.placement = []
    s.append(sharding)
    try:
        yield
    finally:
        s.pop()


def donated_ids() -> set:
    s = getattr(_TLS, "donated", None)
    if s is None:
        s = _TLS.donated = set()
    return s


@contextmanager
def donating(tensor_ids):
    """Tensors (by ``id``) the running jitted function may update in place (``donate_argnums``)."""
    prev = getattr(_TLS, "donated", None)
    _TLS.donated = set(tensor_ids) | (prev or set())
    try:
        yield
    finally:
        _TLS.donated = prev


def is_donated(t) -> bool:
    s = getattr(_TLS, "donated", None)
    return bool(s) and id(t) in s


def in_user_code() -> bool:
    """True while a jitted function's own body runs (not the jit's argument / output handling)."""
    return getattr(_TLS, "user", 0) > 0


@contextmanager
def user_code():
    _TLS.user = getattr(_TLS, "user", 0) + 1
    try:
        yield
    finally:
        _TLS.user -= 1
