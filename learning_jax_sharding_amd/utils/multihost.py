"""Multi-process helpers (one process per GPU).

``process_allgather`` assembles a global array on every process: each process
writes the tiles it is the *first* holder of into a zero buffer and the buffers
are summed with one all-reduce.  Debug/inspection path only; the hot path never
materialises global arrays.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..runtime.devices import process_index

__all__ = ["process_allgather", "sync_global_devices", "broadcast_one_to_all"]


def process_allgather(arr, device: Optional[torch.device] = None) -> torch.Tensor:
    ta = arr.tile
    local_dev = next(iter(arr.local.values())).device if arr.local else torch.device("cpu")
    acc_dtype = torch.float32 if arr.dtype in (torch.bfloat16, torch.float16) else arr.dtype
    buf = torch.zeros(arr.shape, dtype=acc_dtype, device=local_dev)
    for d, t in arr.local.items():
        tile = ta.coords[d]
        if min(ta.holders(tile)) == d:
            buf[ta.indices(d, arr.shape)] = t.detach().to(acc_dtype)
    if dist.is_initialized():
        dist.all_reduce(buf)
    out = buf.to(arr.dtype)
    return out.to(device or torch.device("cpu"))


def sync_global_devices(name: str = "") -> None:
    if dist.is_initialized():
        dist.barrier()


def broadcast_one_to_all(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if dist.is_initialized():
        dist.broadcast(t, src)
    return t
