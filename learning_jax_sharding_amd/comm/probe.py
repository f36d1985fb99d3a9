"""Timed eager all-reduce through every collective path this job can use (bench.py comm_detail).

A multi-GPU benchmark record should say which collective implementation carried its gradients
and what that implementation costs on this node, measured, not assumed.  :func:`all_reduce_paths`
times ONE message size (the step's gradient bytes) through each available path, eagerly, before
the timed region:

* ``rccl``       - the native RCCL world communicator (``comm/native.RankRccl``: ncclAllReduce on
  the current HIP stream, what the captured training step uses);
* ``p2p``        - the peer-memory kernels over IPC-mapped xGMI buffers (``comm/p2p.P2PGroup``,
  one-shot up to ``LJS_P2P_ONESHOT_KB``, two-shot above), with a group built for this size;
* ``torch-<be>`` - ``torch.distributed.all_reduce`` on the default process group (RCCL through
  torch's ``nccl`` backend on GPUs, gloo on CPU ranks).

Every rank calls it at the same point with the same size (it is collective).  Paths that cannot
run here are listed with the reason instead of a time.
"""
from __future__ import annotations

import time
from typing import Dict, List

import torch
import torch.distributed as dist

__all__ = ["all_reduce_paths"]


def _timed(fn, iters: int, warm: int, cuda: bool) -> float:
    for _ in range(warm):
        fn()
    if cuda:
        torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    if cuda:
        torch.cuda.synchronize()
    t = time.perf_counter() - t0
    # the slowest rank sets a collective's time
    tt = torch.tensor([t], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item()) / iters


def _entry(path: str, nbytes: int, n: int, sec: float) -> Dict:
    alg = nbytes / sec / 1e9
    return {"path": path, "bytes": nbytes, "us_per_call": round(sec * 1e6, 2), "algbw_GBps": round(alg, 2),
            "busbw_GBps": round(alg * 2 * (n - 1) / n, 2)}


def all_reduce_paths(nbytes: int, iters: int = 10, warm: int = 3) -> List[Dict]:
    """Time an f32 all-reduce of ``nbytes`` over the world group through each path (see module)."""
    from .backend import get_comm
    from . import p2p
    n = dist.get_world_size()
    comm = get_comm()
    nccl = dist.get_backend() == "nccl"
    cuda = nccl and torch.cuda.is_available()
    dev = torch.device("cuda", torch.cuda.current_device()) if cuda else torch.device("cpu")
    numel = max(4, nbytes // 4 // 4 * 4)
    nbytes = numel * 4
    x = torch.ones(numel, dtype=torch.float32, device=dev)
    out: List[Dict] = []

    nat = getattr(comm, "_native", None)
    if nat is not None:
        h = nat.partition((tuple(range(n)),))
        out.append(_entry("rccl", nbytes, n, _timed(lambda: nat.all_reduce_(h, x), iters, warm, cuda)))
    else:
        out.append({"path": "rccl", "bytes": nbytes, "skipped": "no native RCCL communicator on this backend"})

    if not cuda:
        out.append({"path": "p2p", "bytes": nbytes, "skipped": "peer-memory kernels need distinct GPUs"})
    elif not p2p.enabled() or getattr(comm, "_p2p_off", None):
        out.append({"path": "p2p", "bytes": nbytes, "skipped": getattr(comm, "_p2p_off", None) or "LJS_P2P=0"})
    elif nbytes % (16 * n):
        out.append({"path": "p2p", "bytes": nbytes, "skipped": "size not a multiple of 16 x ranks"})
    else:
        me = dist.get_rank()
        devs = [dev if r == me else torch.device("cuda", 0) for r in range(n)]
        try:
            grp = p2p.P2PGroup(devs, nbytes, rank=me, pg=dist.group.WORLD)
        except p2p.P2PUnavailable as e:
            out.append({"path": "p2p", "bytes": nbytes, "skipped": f"group build failed: {e}"[:200]})
        else:
            y = torch.empty_like(x)
            kind = "p2p-oneshot" if nbytes <= grp.oneshot_max else "p2p-twoshot"
            try:
                ent = _entry(kind, nbytes, n, _timed(lambda: grp.all_reduce({me: x}, out={me: y}), iters, warm, cuda))
                grp.check_error()
                out.append(ent)
            except RuntimeError as e:
                out.append({"path": kind, "bytes": nbytes, "skipped": f"barrier error: {e}"[:200]})
            grp.close()

    pg_x = x if (cuda or not x.is_cuda) else x.cpu()
    out.append(_entry(f"torch-{dist.get_backend()}", nbytes, n,
                      _timed(lambda: dist.all_reduce(pg_x), iters, warm, cuda)))
    return out
