"""bf16 "shadow" copies of f32 parameters for the MFMA GEMMs.

The reference keeps f32 parameters and casts them to bf16 inside every Dense call
(``case6_attention.py:46``, flax ``promote_dtype``).  On MI355X each such cast is a separate
memory-bound kernel per weight per step.  Instead each f32 weight gets persistent bf16
shadows - ``"T"`` (transposed, ``[out][in]``, the k-contiguous B operand of the forward
GEMM) and ``"N"`` (plain ``[in][out]``, used by the backward input-gradient GEMM) - which
the fused multi-tensor Adam kernel rewrites in the same pass that updates the weight.  A
shadow is trusted only while the weight tensor object is alive and its autograd version
counter matches, so any other in-place write to the weight forces a re-cast.
"""
from __future__ import annotations

import weakref
from typing import Dict, Optional

import torch

__all__ = ["get", "entry", "mark_fresh", "kinds_of"]


class _Entry:
    __slots__ = ("ref", "bufs", "versions", "__weakref__")

    def __init__(self, w: torch.Tensor):
        self.ref = weakref.ref(w)
        self.bufs: Dict[str, torch.Tensor] = {}
        self.versions: Dict[str, int] = {}


_REG: Dict[int, _Entry] = {}


def entry(w: torch.Tensor, create: bool = True) -> Optional[_Entry]:
    e = _REG.get(id(w))
    if e is not None and e.ref() is not w:
        e = None
        _REG.pop(id(w), None)
    if e is None and create:
        e = _Entry(w)
        _REG[id(w)] = e
        weakref.finalize(w, _REG.pop, id(w), None)
    return e


def kinds_of(w: torch.Tensor):
    e = entry(w, create=False)
    return {} if e is None else e.bufs


def _alloc(w: torch.Tensor, kind: str) -> torch.Tensor:
    K, N = w.shape
    shape = (N, K) if kind == "T" else (K, N)
    return torch.empty(shape, dtype=torch.bfloat16, device=w.device)


def get(w: torch.Tensor, kind: str) -> torch.Tensor:
    """bf16 copy of the 2-D f32 weight ``w`` (``kind`` "T": transposed, "N": plain)."""
    from . import hip
    e = entry(w)
    buf = e.bufs.get(kind)
    if buf is None:
        buf = e.bufs[kind] = _alloc(w, kind)
        e.versions[kind] = -1
    if e.versions.get(kind) != w._version:
        if kind == "T":
            hip.cast_transpose_bf16(w, buf)
        else:
            buf.copy_(hip._cast_raw(w.contiguous(), torch.bfloat16))
        e.versions[kind] = w._version
    return buf


def mark_fresh(w: torch.Tensor) -> None:
    """Called after a kernel rewrote ``w`` in place AND refreshed all its shadows."""
    torch.autograd.graph.increment_version(w)
    e = entry(w, create=False)
    if e is not None:
        for k in e.bufs:
            e.versions[k] = w._version
