"""Parallelism strategies as first-class components.

* :mod:`.data` - data parallelism: bucketed, backward-overlapped gradient all-reduce;
* :mod:`.fsdp` - fully-sharded data parallelism: FSDP shardings, side-stream prefetched
  parameter all-gathers (their transposes are the overlapped gradient reduce-scatters);
* :mod:`.tensor` - tensor parallelism: rule presets (reference, FSDP, GSPMD "2D finalized", Megatron)
  and explicit column/row-parallel dense layers;
* :mod:`.sequence` - sequence / context parallelism: all-gather-KV and ring attention.

The partitioner (``spmd/``) lowers any of these layouts from sharding annotations; these
modules add the scheduling (overlap, prefetch, ring pipelining) and the presets.
"""
from . import data, fsdp, sequence, tensor  # noqa: F401
from .tensor import PRESETS, rules  # noqa: F401
