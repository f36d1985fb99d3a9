"""Weight gradients on a side HIP stream, overlapping the rest of the backward pass.

A dense layer's weight gradient (``dW = X^T dY``: a split-K slab GEMM plus its reduction) is
needed by nothing else in the backward pass - only by the optimizer afterwards - while the input
gradient ``dX`` feeds the next layer's backward.  Inside :func:`wgrad_scope` (entered by
``value_and_grad`` when no data-parallel gradient hooks watch the backward) every dW is forked
onto a per-device side stream: the main stream records an event the side stream waits for (dY
and X are ready), the dW kernels run on the side stream while the main stream continues with
dX and the layers below, and the scope's exit joins every fork back into the main stream before
the gradients are returned.  Under HIP-graph capture the event record / wait pairs become graph
edges, so the replayed step keeps the concurrency (reference shape: the out-projection's dW
runs beside the attention backward instead of after it).

Tensors cross streams with ``record_stream`` both ways so the caching allocator never hands a
block to one stream while the other may still use it.

Opt-in (``LJS_SIDE_WGRAD=1``): measured on MI355X it LOSES at every bench shape (case6 B=64
0.246-0.258 -> 0.275 ms, B=8 0.111 -> 0.122 ms, attention+FF layer 0.69 -> 0.77 ms): the
persistent GEMM grids are sized for the whole chip (blocks per CU x CUs, one round), so two of
them sharing the CUs turn one round into two plus a tail, and the concurrent kernels evict
each other's operand panels from L2.  Gradients are bit-identical either way
(``tests/test_epilogue_gpu.py::test_side_stream_weight_grads_bit_exact``).
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, List, Tuple

import torch

__all__ = ["wgrad_scope", "side", "join", "enabled"]

_ENABLED = False
_SIDE: Dict[int, torch.cuda.Stream] = {}
_PENDING: List[Tuple[torch.device, torch.cuda.Event, List[torch.Tensor]]] = []


def enabled() -> bool:
    return _ENABLED


@contextlib.contextmanager
def wgrad_scope(active: bool = True):
    """Weight gradients computed inside go to side streams (when ``active`` and not disabled by
    ``LJS_SIDE_WGRAD=0``); every fork is joined into the main streams on exit."""
    global _ENABLED
    prev = _ENABLED
    _ENABLED = bool(active and os.environ.get("LJS_SIDE_WGRAD", "0") == "1")
    try:
        yield
    finally:
        _ENABLED = prev
        join()


@contextlib.contextmanager
def side(dev: torch.device, inputs=()):
    """Run the body on ``dev``'s side stream after the work queued so far on its current stream;
    append the tensors the body produces to the yielded list (they are handed back to the main
    stream at the join).  Outside :func:`wgrad_scope` (or on host devices) the body runs inline."""
    if not _ENABLED or dev.type != "cuda":
        yield []
        return
    main = torch.cuda.current_stream(dev)
    s = _SIDE.get(dev.index)
    if s is None:
        s = _SIDE[dev.index] = torch.cuda.Stream(dev)
    ev = torch.cuda.Event()
    ev.record(main)
    s.wait_event(ev)
    for t in inputs:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            t.record_stream(s)
    outs: List[torch.Tensor] = []
    with torch.cuda.stream(s):
        yield outs
    done = torch.cuda.Event()
    done.record(s)
    _PENDING.append((dev, done, outs))


def join() -> None:
    """The main stream of every device with pending side work waits for it."""
    while _PENDING:
        dev, ev, outs = _PENDING.pop(0)
        main = torch.cuda.current_stream(dev)
        main.wait_event(ev)
        for t in outs:
            if isinstance(t, torch.Tensor):
                t.record_stream(main)
