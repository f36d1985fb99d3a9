"""bf16 "shadow" copies of f32 parameters for the MFMA GEMMs.

The reference keeps f32 parameters and casts them to bf16 inside every Dense call
(``case6_attention.py:46``, flax ``promote_dtype``).  On MI355X each such cast is a separate
memory-bound kernel per weight per step.  Instead each f32 weight gets persistent bf16
shadows - ``"T"`` (transposed, ``[out][in]``, the k-contiguous B operand of the forward
GEMM) and ``"N"`` (plain ``[in][out]``, used by the backward input-gradient GEMM) - which
the fused multi-tensor Adam kernel rewrites in the same pass that updates the weight.

Keying: by storage address + layout, validated by (a) a weak reference to the tensor that
owns the storage (the optimizer's parameter; while it lives the address cannot be reused)
and (b) torch's version counter, which ``detach()`` views share with their base - so the
autograd leaves ``grad`` creates for a step hit the same shadow, and any in-place write
that is not the fused optimizer forces a re-cast.
"""
from __future__ import annotations

import weakref
from typing import Dict, List, Optional, Sequence, Tuple

import torch

__all__ = ["get", "get_stacked", "get_mx", "mx_eligible", "entry", "adopt", "mark_fresh", "kinds_of", "register_proxy",
           "register_mx_proxy", "is_proxy"]


class _Entry:
    __slots__ = ("ref", "bufs", "versions", "proxy", "shared", "mx")

    def __init__(self, w: torch.Tensor):
        self.ref = weakref.ref(w)
        self.bufs: Dict[str, torch.Tensor] = {}
        self.versions: Dict[str, int] = {}
        self.proxy = False
        self.shared = None   # proxies of ONE gathered buffer (virtual devices of a GPU): derived shadows
        self.mx = None       # MX-fp8 proxies: {"QT": (q, s), "QN": (q, s)} gathered from the shards


_REG: Dict[Tuple, _Entry] = {}
import os as _os
_TRACE = _os.environ.get("LJS_SHADOW_TRACE", "0") == "1"


def _key(w: torch.Tensor):
    return (w.data_ptr(), w.dtype, tuple(w.shape), tuple(w.stride()), w.device)


def _owner_of(w: torch.Tensor) -> torch.Tensor:
    """The persistent tensor whose storage ``w`` views: the parameter an autograd leaf was
    detached from (``spmd.api._fresh_leaf`` records it), else ``w`` itself.  Shadows are owned by
    it, so they survive the per-step leaves (a sharded weight's shadow would otherwise be re-cast
    every step once the leaf is gone before the optimizer adopts it)."""
    b = getattr(w, "_ljs_base", None)
    return b if b is not None and b.data_ptr() == w.data_ptr() else w


def entry(w: torch.Tensor, create: bool = True) -> Optional[_Entry]:
    k = _key(w)
    e = _REG.get(k)
    if e is not None:
        owner = e.ref()
        if owner is None or owner.data_ptr() != w.data_ptr():
            e = None
            _REG.pop(k, None)
    if e is None and create:
        e = _Entry(_owner_of(w))
        _REG[k] = e
    return e


def adopt(w: torch.Tensor) -> Optional[_Entry]:
    """The optimizer's parameter tensor becomes the owner of its storage's shadows."""
    e = entry(w, create=False)
    if e is not None and e.ref() is not w:
        e.ref = weakref.ref(w)
    return e


def kinds_of(w: torch.Tensor):
    e = adopt(w)
    return {} if e is None else e.bufs


def _alloc(w: torch.Tensor, kind: str) -> torch.Tensor:
    K, N = w.shape
    shape = (N, K) if kind == "T" else (K, N)
    return torch.empty(shape, dtype=torch.bfloat16, device=w.device)


def _refresh(w: torch.Tensor, e: _Entry, kind: str) -> torch.Tensor:
    from . import hip
    buf = e.bufs[kind]
    if e.proxy:
        if e.versions.get(kind) != w._version:
            if kind == "N" and "T" in e.bufs and e.versions.get("T") == w._version:
                hip.transpose_bf16(e.bufs["T"], buf)     # derived from the gathered [out][in] shadow
                e.versions[kind] = w._version
                if e.shared is not None:
                    e.shared[kind] = buf
            else:
                raise RuntimeError("shadow of a gathered-weight proxy requested that cannot be derived from its "
                                   f"gathered bf16 copy (kind {kind!r}); the proxy holds no f32 values")
        return buf
    if e.versions.get(kind) != w._version:
        if _TRACE:
            import sys
            print(f"[shadow] refresh {kind} {tuple(w.shape)} ptr={w.data_ptr():#x} ver={w._version} "
                  f"had={e.versions.get(kind)} owner_alive={e.ref() is not None}", file=sys.stderr)
        if kind == "T":
            hip.cast_transpose_bf16(w, buf)
        else:
            hip._cast_raw(w.contiguous(), torch.bfloat16, out=buf)   # cast straight into the shadow
        e.versions[kind] = w._version
    return buf


def get(w: torch.Tensor, kind: str) -> torch.Tensor:
    """bf16 copy of the 2-D f32 weight ``w`` (``kind`` "T": transposed, "N": plain)."""
    e = entry(w)
    if e.proxy and e.shared is not None and kind in e.shared:
        return e.shared[kind]                 # derived once for every proxy sharing the buffer
    if kind not in e.bufs:
        e.bufs[kind] = _alloc(w, kind)
        e.versions[kind] = -1
    return _refresh(w, e, kind)


def stacked_proxy_T(ws: Sequence[torch.Tensor]) -> bool:
    """Whether same-shape proxies' "T" shadows already sit in consecutive slices of one buffer."""
    es = [entry(w, create=False) for w in ws]
    if any(e is None or not e.proxy or "T" not in e.bufs for e in es):
        return False
    K, N = ws[0].shape
    base = es[0].bufs["T"]
    return all(e.bufs["T"].data_ptr() == base.data_ptr() + i * N * K * 2 for i, e in enumerate(es))


def register_proxy(w: torch.Tensor, t_buf: torch.Tensor, shared: Optional[dict] = None) -> None:
    """``w`` (an uninitialised f32 tensor of the full weight's shape) stands for a weight whose bf16
    transposed shadow ``t_buf`` [out][in] was all-gathered from the shards' own shadows
    (parallel/weight_gather.py): the GEMMs read ``t_buf`` (and an "N" shadow transposed from it);
    asking for anything that needs the f32 values raises.  ``shared``: one dict for all the
    proxies standing for the same ``t_buf`` (virtual devices of one GPU): shadows derived from it
    are computed once."""
    e = entry(w)
    e.proxy = True
    e.shared = shared
    e.bufs["T"] = t_buf
    e.versions["T"] = w._version
    # the entry (and the gathered buffers it holds) goes with the proxy
    weakref.finalize(w, _drop, _key(w), e)


def _drop(key, e) -> None:
    if _REG.get(key) is e:
        del _REG[key]


def is_proxy(w: torch.Tensor) -> bool:
    e = entry(w, create=False)
    return e is not None and e.proxy


def register_mx_proxy(w: torch.Tensor, mx: Dict[str, Tuple[torch.Tensor, torch.Tensor]]) -> None:
    """``w`` (an uninitialised f32 tensor of the full weight's shape) stands for a weight whose
    MX-fp8 shadows ``mx`` ("QT" and "QN": (codes, scales)) were all-gathered from the shards' own
    (``parallel/weight_gather.gather_mx``): the MX GEMMs read them; anything needing the f32
    values or a bf16 shadow raises."""
    e = entry(w)
    e.proxy = True
    e.mx = dict(mx)
    weakref.finalize(w, _drop, _key(w), e)


def mx_eligible(w: torch.Tensor) -> bool:
    """Weights whose MX-fp8 shadows the fused Adam can keep (64 x 64 tiles of its 4-wide path;
    a launch carrying MX shadows always runs 64-row tiles unless a test forces another height)."""
    from . import hip
    return (w.is_cuda and w.dim() == 2 and w.dtype == torch.float32 and w.is_contiguous()
            and w.shape[0] % 64 == 0 and w.shape[1] % 64 == 0 and hip.adam_rows() in (0, 64))


def get_mx(w: torch.Tensor, kind: str):
    """(q, s) MX-fp8 shadow of the f32 weight ``w`` [K][N]: ``"QT"`` = q [N][K] with scales
    [N][K/32] (blocks along K: a forward GEMM's B operand, ``fp8.quant_cols``), ``"QN"`` = q [K][N]
    with scales [K][N/32] (blocks along N: a dX GEMM's B operand, ``fp8.quant_rows``).  The fused
    Adam rewrites them with the weight (``hip.adam_multi``); any other write re-quantizes."""
    from . import fp8
    e = entry(w)
    if e.proxy:
        if e.mx is not None and kind in e.mx:
            return e.mx[kind]
        raise RuntimeError("MX-fp8 shadows of a gathered-weight proxy are not available (bf16 gather)")
    K, N = w.shape
    if kind not in e.bufs:
        qs = (N, K) if kind == "QT" else (K, N)
        e.bufs[kind] = torch.empty(qs, dtype=torch.uint8, device=w.device)
        e.bufs[kind + "s"] = torch.empty((qs[0], qs[1] // 32), dtype=torch.uint8, device=w.device)
        e.versions[kind] = -1
    q, s = e.bufs[kind], e.bufs[kind + "s"]
    if e.versions.get(kind) != w._version:
        if kind == "QT":
            fp8.quant_cols(w, out=(q, s))
        else:
            fp8.quant_rows(w, out=(q, s))
        e.versions[kind] = e.versions[kind + "s"] = w._version
    return q, s


def get_stacked(ws: Sequence[torch.Tensor]) -> torch.Tensor:
    """``[n][N][K]`` transposed shadows of same-shape weights as ONE buffer (batched GEMM operand).

    The first call moves the weights' "T" shadows into consecutive slices of one allocation;
    the fused Adam then writes them there directly, so no per-step stacking copy remains.
    """
    es = [entry(w) for w in ws]
    K, N = ws[0].shape
    if any(e.proxy for e in es) and not stacked_proxy_T(ws):
        raise RuntimeError("gathered-weight proxies must arrive stacked (one gather of the stacked shadows)")
    bufs = [e.bufs.get("T") for e in es]
    base = bufs[0]
    ok = all(b is not None for b in bufs) and base is not None and all(
        b.data_ptr() == base.data_ptr() + i * N * K * 2 for i, b in enumerate(bufs))
    if not ok:
        group = torch.empty((len(ws), N, K), dtype=torch.bfloat16, device=ws[0].device)
        for i, (w, e) in enumerate(zip(ws, es)):
            old = e.bufs.get("T")
            e.bufs["T"] = group[i]
            if old is not None and e.versions.get("T") == w._version:
                group[i].copy_(old)
            else:
                e.versions["T"] = -1
    for w, e in zip(ws, es):
        _refresh(w, e, "T")
    b0 = es[0].bufs["T"]
    return b0.as_strided((len(ws), N, K), (N * K, K, 1))


def mark_fresh(w: torch.Tensor) -> None:
    """Called after a kernel rewrote ``w`` in place AND refreshed all its shadows."""
    torch.autograd.graph.increment_version(w)
    e = entry(w, create=False)
    if e is not None:
        for k in e.bufs:
            e.versions[k] = w._version
