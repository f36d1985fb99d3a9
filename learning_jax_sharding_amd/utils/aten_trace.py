"""Which torch (aten) kernels does a step still launch, and from where?

Every hot op of the framework is a hand-written HIP kernel called through ctypes; anything
that still reaches PyTorch's own kernels (``at::native`` copies, cats, adds, fills - the
``__amd_rocclr_copyBuffer`` / ``elementwise_kernel`` rows of a rocprof table) goes through the
aten dispatcher.  :class:`AtenTrace` is a ``TorchDispatchMode`` that records each such call
with the framework frames of its Python stack, so a profile row can be traced to its call site.

Views, allocations and metadata ops launch nothing and are skipped.  Used by
``bench.py`` when ``LJS_ATEN_TRACE=<file>`` is set (one extra un-captured step is traced after
the warm-up; the timed steps are untouched).
"""
from __future__ import annotations

import collections
import os
import traceback
from typing import Dict, List, Tuple

import torch
from torch.utils._python_dispatch import TorchDispatchMode

# ops that launch no kernel
_FREE = {
    "view", "_unsafe_view", "reshape", "permute", "as_strided", "t", "transpose", "expand", "slice", "select",
    "squeeze", "unsqueeze", "detach", "alias", "empty", "empty_strided", "empty_like", "new_empty",
    "new_empty_strided", "split", "split_with_sizes", "chunk", "unbind", "narrow", "view_as_real",
    "view_as_complex", "lift_fresh", "_reshape_alias", "movedim", "unflatten", "flatten", "sym_size",
    "sym_stride", "sym_numel", "sym_storage_offset", "is_same_size", "_local_scalar_dense", "item",
    "set_", "resize_", "record_stream", "is_pinned", "_has_compatible_shallow_copy_type", "dim",
    "size", "stride", "storage_offset", "numel", "is_contiguous", "diagonal",
}

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_ROOT = os.path.dirname(_PKG)


def _site(depth: int = 4) -> Tuple[str, ...]:
    """The innermost ``depth`` framework frames of the current stack; when the innermost Python
    frame is outside the framework (torch's autograd / dispatch code), it leads as ``[torch] ...``
    so an op launched from inside torch (e.g. an autograd Function's output handling) is told
    apart from one the framework line issued itself."""
    out = []
    first = True
    for fr in reversed(traceback.extract_stack()[:-3]):
        f = os.path.abspath(fr.filename)
        if "aten_trace" in f or "_python_dispatch" in f:
            continue
        if f.startswith(_ROOT):
            out.append(f"{os.path.relpath(f, _ROOT)}:{fr.lineno} {fr.name}")
            if len(out) >= depth:
                break
        elif first:
            out.append(f"[torch] {os.path.basename(f)}:{fr.lineno} {fr.name}")
        first = False
    return tuple(out)


def _desc(a) -> str:
    if isinstance(a, torch.Tensor):
        return f"{str(a.dtype).replace('torch.', '')}{list(a.shape)}"
    if isinstance(a, (list, tuple)) and a and isinstance(a[0], torch.Tensor):
        return f"[{len(a)}x {_desc(a[0])}]"
    return ""


# framework (ops.hip) helpers whose launches are data movement or glue rather than the step's
# math: traced by call site too (they are ctypes calls, invisible to the dispatcher)
_HIP_GLUE = ("rank_major", "from_rank_major", "concat_parts", "slab_reduce", "cast_transpose_bf16", "swap01_bf16",
             "transpose_bf16", "colsum_ld", "sum_n", "sum_ptrs", "cast", "cast_into", "bcast_scalar", "pad_box",
             "_pack_launch")


class AtenTrace(TorchDispatchMode):
    """Record kernel-launching aten calls (and the framework's glue kernels, ``_HIP_GLUE``):
    ``(op, operand shapes, call site) -> count``."""

    def __init__(self, cuda_only: bool = True, depth: int = 6):
        super().__init__()
        self.cuda_only = cuda_only
        self.depth = depth
        self.calls: Dict[Tuple[str, str, Tuple[str, ...]], int] = collections.Counter()
        self._saved = {}

    def __enter__(self):
        from ..ops import hip
        for name in _HIP_GLUE:
            fn = getattr(hip, name, None)
            if fn is None:
                continue
            self._saved[name] = fn

            def wrap(*a, _fn=fn, _name=name, **k):
                shapes = " ".join(s for s in (_desc(x) for x in a) if s)
                self.calls[("hip." + _name, shapes, _site(self.depth))] += 1
                return _fn(*a, **k)
            setattr(hip, name, wrap)
        return super().__enter__()

    def __exit__(self, *exc):
        from ..ops import hip
        for name, fn in self._saved.items():
            setattr(hip, name, fn)
        self._saved.clear()
        return super().__exit__(*exc)

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = func.overloadpacket.__name__
        if name not in _FREE:
            ts = [a for a in list(args) + list(kwargs.values()) if isinstance(a, torch.Tensor)]
            ts += [t for a in args if isinstance(a, (list, tuple)) for t in a if isinstance(t, torch.Tensor)]
            if not self.cuda_only or any(t.is_cuda for t in ts) or kwargs.get("device") is not None:
                shapes = " ".join(s for s in (_desc(a) for a in args) if s)
                self.calls[(str(func), shapes, _site(self.depth))] += 1
        return func(*args, **(kwargs or {}))

    def report(self) -> List[str]:
        lines = [f"{len(self.calls)} distinct aten call sites, {sum(self.calls.values())} calls"]
        for (op, shapes, site), n in sorted(self.calls.items(), key=lambda kv: -kv[1]):
            lines.append(f"{n:4d}  {op}  {shapes}")
            for s in site:
                lines.append(f"        {s}")
        return lines

    def write(self, path: str) -> None:
        with open(path, "w") as f:
            f.write("\n".join(self.report()) + "\n")
