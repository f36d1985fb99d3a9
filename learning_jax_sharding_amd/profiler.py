"""Profiling and debugging aids (tracing/profiling, race detection).

* :func:`annotate` - named ranges (roctx markers through torch's nvtx shim on ROCm) that
  ``rocprofv3 --marker-trace`` shows around the partitioner's ops;
* :class:`StepTimer` - HIP-event timing of steps (median / p90 / mean), no host sync inside
  the timed region;
* :func:`collective_plan` - the printable collective plan of a function (what GSPMD's HLO
  dump is to the reference);
* debug modes (env, read at call time):
    ``LJS_DEBUG_SYNC=1``   synchronise after every HIP kernel launch and every collective, so
                           an asynchronous fault is reported at the op that caused it (the
                           "fully-synchronous execution" half of an async/sync comparison);
    ``LJS_DEBUG_NANS=1``   check every collective's output for NaN/Inf and raise at the first;
  :func:`compare_sync_async` runs a step function both ways and reports the max difference
  (stream-ordering races show up as differences).
"""
from __future__ import annotations

import contextlib
import os
import statistics
from typing import Any, Callable, Dict, List, Optional

import torch

__all__ = ["annotate", "StepTimer", "collective_plan", "debug_sync_enabled", "debug_nans_enabled",
           "after_kernel", "after_collective", "compare_sync_async", "rocprof_command"]


def debug_sync_enabled() -> bool:
    return os.environ.get("LJS_DEBUG_SYNC", "0") == "1"


def debug_nans_enabled() -> bool:
    return os.environ.get("LJS_DEBUG_NANS", "0") == "1"


@contextlib.contextmanager
def annotate(name: str):
    """A named range visible in rocprofv3 marker traces (no-op without a GPU)."""
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield


def after_kernel(name: str) -> None:
    """Called by the HIP launchers after a launch; synchronises in LJS_DEBUG_SYNC mode."""
    if debug_sync_enabled() and torch.cuda.is_available():
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:  # pragma: no cover - only on a faulting kernel
            raise RuntimeError(f"HIP fault surfaced after kernel {name}: {e}") from e


def after_collective(kind: str, out: Dict[int, torch.Tensor]) -> None:
    if debug_sync_enabled() and torch.cuda.is_available():
        torch.cuda.synchronize()
    if debug_nans_enabled():
        for d, t in out.items():
            if t.is_floating_point() and not bool(torch.isfinite(t).all()):
                raise FloatingPointError(f"non-finite values after {kind} on device {d}")


class StepTimer:
    """Times repeated calls with HIP events (falls back to wall clock on CPU)."""

    def __init__(self):
        self.ms: List[float] = []

    def time(self, fn: Callable[[], Any], steps: int = 10, warmup: int = 2) -> "StepTimer":
        for _ in range(warmup):
            fn()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
            for s, e in evs:
                s.record()
                fn()
                e.record()
            torch.cuda.synchronize()
            self.ms += [s.elapsed_time(e) for s, e in evs]
        else:
            import time
            for _ in range(steps):
                t0 = time.perf_counter()
                fn()
                self.ms.append((time.perf_counter() - t0) * 1e3)
        return self

    def summary(self) -> Dict[str, float]:
        xs = sorted(self.ms)
        return {"median_ms": statistics.median(xs), "p90_ms": xs[int(0.9 * (len(xs) - 1))],
                "mean_ms": statistics.fmean(xs), "n": len(xs)}


def collective_plan(fn: Callable, *args, **kwargs) -> str:
    """The partitioned program's collective plan (``jit(fn).lower(*args).as_text()``)."""
    from .spmd.api import jit
    return jit(fn).lower(*args, **kwargs).as_text()


def compare_sync_async(step: Callable[[], Any], extract: Callable[[Any], List[Any]]) -> float:
    """Run ``step`` asynchronously and with LJS_DEBUG_SYNC, return the max abs difference of
    ``extract(result)`` (0 for a race-free, deterministic program)."""
    import numpy as np
    a = [np.asarray(x, dtype=np.float64) for x in extract(step())]
    old = os.environ.get("LJS_DEBUG_SYNC")
    os.environ["LJS_DEBUG_SYNC"] = "1"
    try:
        b = [np.asarray(x, dtype=np.float64) for x in extract(step())]
    finally:
        if old is None:
            os.environ.pop("LJS_DEBUG_SYNC", None)
        else:
            os.environ["LJS_DEBUG_SYNC"] = old
    return max((float(np.abs(x - y).max()) for x, y in zip(a, b)), default=0.0)


def rocprof_command(cmd: List[str], out_dir: str, counters: Optional[List[str]] = None) -> List[str]:
    """The rocprofv3 invocation used for this repo's profiles: kernel trace + stats, or a
    counter pass (never combined with runtime/marker tracing)."""
    base = ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", out_dir]
    if counters:
        base = ["rocprofv3", "--kernel-trace", "--pmc", *counters, "--output-format", "csv", "-d", out_dir]
    return base + ["--"] + list(cmd)
