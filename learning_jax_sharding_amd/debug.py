"""``jax.debug`` subset: ``visualize_array_sharding`` / ``visualize_sharding`` (``case1b.py:26``,
``case5_attention_dense.py:91``), ``print`` and ``callback``.

Execution is eager, so ``print`` / ``callback`` run when reached, with the global values of
sharded arguments gathered to the host (``numpy.asarray``); inside a captured step
(``jit(capture=True)``) they run once, at capture, like a trace-time print - use them outside
captured steps, or with ``LJS_DEBUG_SYNC=1``.  In multi-process runs only process 0 prints
(``jax.debug.print`` prints once per device; one line per job is the readable form here)."""
from __future__ import annotations

import builtins
from typing import Any, Callable

from .utils.visualize import visualize_array_sharding, visualize_sharding  # noqa: F401

__all__ = ["visualize_array_sharding", "visualize_sharding", "print", "callback"]


def _host(x: Any) -> Any:
    from .array import ShardedArray
    from .utils.tree import tree_map
    import numpy as np
    return tree_map(lambda a: np.asarray(a) if isinstance(a, ShardedArray) else a, x)


def callback(fn: Callable[..., Any], *args: Any, **kwargs: Any) -> None:
    """``jax.debug.callback``: call ``fn`` with the host values of ``args`` / ``kwargs``."""
    fn(*_host(list(args)), **_host(dict(kwargs)))


def print(fmt: str, *args: Any, **kwargs: Any) -> None:  # noqa: A001 - jax.debug.print
    """``jax.debug.print``: ``fmt.format(*args, **kwargs)`` on the host values (process 0)."""
    from .runtime.devices import process_index
    if process_index() != 0:
        return
    builtins.print(fmt.format(*_host(list(args)), **_host(dict(kwargs))))
