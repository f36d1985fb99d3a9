"""Single-controller RCCL over xGMI through the native runtime (``_lib/libljs_runtime.so``,
``csrc/runtime/comm.cpp``).

One Python process driving several physical MI355X (the JAX-like single-controller mode of
SURVEY §2.5/§7) issues every collective of a device group for all members inside one
``ncclGroupStart/End``, each member on its own current HIP stream.  Communicators come from
``ncclCommInitAll`` and are cached per ordered tuple of physical GPUs.  Groups containing
the same GPU twice (virtual devices) are not eligible: the copy-based loopback path of
:class:`~.backend.LocalComm` serves them.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Dict, Optional, Sequence, Tuple

import torch

__all__ = ["available", "runtime", "device_info", "eligible", "NativeRccl", "RankRccl", "rank_eligible"]

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIBPATH = os.path.join(os.path.dirname(_HERE), "_lib", "libljs_runtime.so")
_LIB = None
_LOCK = threading.Lock()
_VP = ctypes.c_void_p

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int32: 3, torch.int64: 4, torch.uint8: 5}


def runtime():
    global _LIB
    if _LIB is None:
        with _LOCK:
            if _LIB is None:
                if not os.path.exists(_LIBPATH):
                    raise RuntimeError(f"native runtime not built: {_LIBPATH} (run csrc/build.py)")
                L = ctypes.CDLL(_LIBPATH)
                sig = {
                    "ljs_rt_version": [],
                    "ljs_rt_device_info": [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_long)],
                    "ljs_comm_init": [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(_VP)],
                    "ljs_comm_destroy": [_VP],
                    "ljs_comm_all_reduce": [_VP, ctypes.POINTER(_VP), ctypes.POINTER(_VP), ctypes.c_size_t, ctypes.c_int,
                                            ctypes.c_int, ctypes.POINTER(_VP)],
                    "ljs_comm_all_gather": [_VP, ctypes.POINTER(_VP), ctypes.POINTER(_VP), ctypes.c_size_t, ctypes.c_int,
                                            ctypes.POINTER(_VP)],
                    "ljs_comm_reduce_scatter": [_VP, ctypes.POINTER(_VP), ctypes.POINTER(_VP), ctypes.c_size_t,
                                                ctypes.c_int, ctypes.c_int, ctypes.POINTER(_VP)],
                    "ljs_comm_all_to_all": [_VP, ctypes.POINTER(_VP), ctypes.POINTER(_VP), ctypes.c_size_t, ctypes.c_int,
                                            ctypes.POINTER(_VP)],
                    "ljs_comm_split": [_VP, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                       ctypes.POINTER(_VP)],
                    "ljs_comm_async_error": [_VP],
                    "ljs_comm_abort": [_VP],
                    "ljs_comm_unique_id_size": [],
                    "ljs_comm_get_unique_id": [ctypes.c_char_p],
                    "ljs_comm_init_rank": [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(_VP)],
                    "ljs_comm_split_rank": [_VP, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_VP)],
                    "ljs_comm_nranks": [_VP],
                    "ljs_comm_query": [_VP, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                       ctypes.POINTER(ctypes.c_int)],
                }
                for name, argt in sig.items():
                    fn = getattr(L, name)
                    fn.argtypes = argt
                    fn.restype = ctypes.c_int
                L.ljs_comm_error_string.argtypes = [ctypes.c_int]
                L.ljs_comm_error_string.restype = ctypes.c_char_p
                _LIB = L
    return _LIB


def available() -> bool:
    try:
        runtime()
        return True
    except (RuntimeError, OSError):
        return False


def device_info(dev: int = 0) -> Dict[str, int]:
    """CU count, LDS per CU, L2 bytes, wavefront size, XCD hint and HBM bytes of a GPU."""
    out = (ctypes.c_int * 5)()
    hbm = ctypes.c_long()
    rc = runtime().ljs_rt_device_info(dev, out, ctypes.byref(hbm))
    if rc:
        raise RuntimeError(f"hipGetDeviceProperties failed: {rc}")
    return {"cus": out[0], "lds_bytes": out[1], "l2_bytes": out[2], "wavefront": out[3], "xcds": out[4],
            "hbm_bytes": hbm.value}


def eligible(devices: Sequence[torch.device]) -> bool:
    if os.environ.get("LJS_NATIVE_RCCL", "1") == "0" or len(devices) < 2:
        return False
    if not all(d.type == "cuda" for d in devices):
        return False
    idx = [d.index for d in devices]
    return len(set(idx)) == len(idx) and available()


def _ptrs(ts):
    return (_VP * len(ts))(*[t.data_ptr() for t in ts])


def _streams(ts):
    return (_VP * len(ts))(*[torch.cuda.current_stream(t.device).cuda_stream for t in ts])


class NativeRccl:
    """Communicator cache + collectives over groups of distinct physical GPUs."""

    def __init__(self):
        self._comms: Dict[Tuple[int, ...], int] = {}
        self._world: Optional[Tuple[int, ...]] = None

    def _init_all(self, gpus: Tuple[int, ...]) -> int:
        arr = (ctypes.c_int * len(gpus))(*gpus)
        out = _VP()
        self._check(runtime().ljs_comm_init(len(gpus), arr, ctypes.byref(out)), "ncclCommInitAll")
        return out.value

    def comm(self, gpus: Tuple[int, ...]) -> int:
        """Communicator of an ordered group of distinct GPUs.  The first one covers every
        visible GPU (the "world"); mesh-axis subgroups are then carved out of it with
        ncclCommSplit, falling back to a fresh ncclCommInitAll."""
        h = self._comms.get(gpus)
        if h is not None:
            return h
        if self._world is None:
            world = tuple(range(torch.cuda.device_count()))
            if set(gpus) <= set(world) and len(world) > len(gpus):
                self._world = world
                self._comms[world] = self._init_all(world)
        world = self._world
        if world is not None and gpus != world and set(gpus) <= set(world):
            colors = (ctypes.c_int * len(world))(*[0 if g in gpus else -1 for g in world])
            keys = (ctypes.c_int * len(world))(*[gpus.index(g) if g in gpus else 0 for g in world])
            out = (_VP * 1)()
            if runtime().ljs_comm_split(self._comms[world], colors, keys, 1, out) == 0:
                h = self._comms[gpus] = out[0]
                return h
        h = self._comms[gpus] = self._init_all(gpus)
        return h

    def check(self) -> None:
        """Failure detection: raise on the first asynchronous RCCL error of any
        cached communicator (ncclCommGetAsyncError)."""
        for gpus, h in self._comms.items():
            rc = runtime().ljs_comm_async_error(h)
            if rc:
                raise RuntimeError(f"RCCL communicator {gpus} failed: {runtime().ljs_comm_error_string(rc).decode()}")

    def wait(self, ts: Sequence[torch.Tensor], timeout_s: float = 60.0) -> None:
        """Wait for the members' streams with a deadline, polling RCCL's async error state; on
        timeout every communicator is aborted and an error raised instead of hanging."""
        import time
        evs = []
        for t in ts:
            e = torch.cuda.Event()
            e.record(torch.cuda.current_stream(t.device))
            evs.append(e)
        t0 = time.time()
        while not all(e.query() for e in evs):
            self.check()
            if time.time() - t0 > timeout_s:
                for h in self._comms.values():
                    runtime().ljs_comm_abort(h)
                self._comms.clear()
                raise TimeoutError(f"collective did not complete within {timeout_s} s; communicators aborted")
            time.sleep(1e-4)

    @staticmethod
    def _check(rc, what):
        if rc:
            raise RuntimeError(f"{what} failed: {runtime().ljs_comm_error_string(rc).decode()}")

    def all_reduce(self, ts: Sequence[torch.Tensor]) -> None:
        """In-place sum over the members' contiguous tensors (member order = list order)."""
        h = self.comm(tuple(t.device.index for t in ts))
        rc = runtime().ljs_comm_all_reduce(h, _ptrs(ts), _ptrs(ts), ts[0].numel(), _DT[ts[0].dtype], 0, _streams(ts))
        self._check(rc, "all_reduce")

    def all_gather(self, ts: Sequence[torch.Tensor]):
        """Returns per member a [n, *shape] tensor of every member's block, member-major."""
        n = len(ts)
        from .backend import _slots_like
        outs = [_slots_like(t, n) for t in ts]
        h = self.comm(tuple(t.device.index for t in ts))
        rc = runtime().ljs_comm_all_gather(h, _ptrs(ts), _ptrs(outs), ts[0].numel(), _DT[ts[0].dtype], _streams(ts))
        self._check(rc, "all_gather")
        return outs

    def reduce_scatter(self, ts: Sequence[torch.Tensor]):
        """ts[i] is [n, *chunk] (chunk r destined to member r); returns each member's summed chunk."""
        outs = [torch.empty_like(t[0]) for t in ts]
        h = self.comm(tuple(t.device.index for t in ts))
        rc = runtime().ljs_comm_reduce_scatter(h, _ptrs(ts), _ptrs(outs), outs[0].numel(), _DT[ts[0].dtype], 0,
                                               _streams(ts))
        self._check(rc, "reduce_scatter")
        return outs

    def all_to_all(self, ts: Sequence[torch.Tensor]):
        """ts[i] is [n, *chunk]; chunk r of member i lands as chunk i of member r."""
        outs = [torch.empty_like(t) for t in ts]
        h = self.comm(tuple(t.device.index for t in ts))
        rc = runtime().ljs_comm_all_to_all(h, _ptrs(ts), _ptrs(outs), ts[0][0].numel(), _DT[ts[0].dtype],
                                           _streams(ts))
        self._check(rc, "all_to_all")
        return outs

    def describe(self):
        return [f"GPU group {list(g)}" for g in self._comms]

    def abort(self) -> None:
        for h in self._comms.values():
            runtime().ljs_comm_abort(h)

    def close(self):
        for h in self._comms.values():
            runtime().ljs_comm_destroy(h)
        self._comms.clear()
        self._world = None


# ============================================================================ one process per GPU
def rank_eligible() -> bool:
    """Native rank communicators for torchrun jobs: RCCL (``nccl``) process group, a GPU, the
    runtime library, and not disabled with ``LJS_NATIVE_RCCL=0``."""
    import torch.distributed as dist
    if os.environ.get("LJS_NATIVE_RCCL", "1") == "0" or not torch.cuda.is_available():
        return False
    if not (dist.is_available() and dist.is_initialized()) or dist.get_backend() != "nccl":
        return False
    return available()


class RankRccl:
    """RCCL communicators of a one-process-per-GPU job, driven through the native runtime.

    The world communicator is created with ``ncclCommInitRank`` from a unique id that rank 0
    publishes in the torch.distributed store; the communicator of every device group of a
    partition is carved out of it with ONE collective ``ncclCommSplit`` per partition (colour
    = the group's index, key = rank order inside the group, so communicator ranks follow sorted
    global ranks like torch process groups).  Every rank must create partitions in the same
    order - the SPMD program guarantees it, as it does for ``dist.new_group``.

    Collectives are plain RCCL calls on the caller's current HIP stream: inside a HIP-graph
    capture they become graph nodes, so a training step with its gradient all-reduces replays
    as ONE graph (no capture cuts, no per-collective Python)."""

    _SEQ = [0]
    _mu = threading.Lock()   # (class default for instances built without __init__: test doubles)

    def __init__(self, rank: int, world: int, device: int):
        self.rank, self.world, self.device = rank, world, device
        self._world_h = self._init_world()
        self._parts: Dict[Tuple[Tuple[int, ...], ...], Optional[int]] = {}
        self._log: Dict[int, Dict[str, Tuple[int, int]]] = {}
        # the watchdog thread (comm/watchdog.py) reads _parts / _log while the main thread adds
        # partitions and collective kinds: both sides go through this lock and readers iterate
        # snapshots
        self._mu = threading.Lock()

    def _init_world(self) -> int:
        import torch.distributed as dist
        store = dist.distributed_c10d._get_default_store()
        RankRccl._SEQ[0] += 1
        key = f"ljs/rccl_uid/{RankRccl._SEQ[0]}"
        n = runtime().ljs_comm_unique_id_size()
        if self.rank == 0:
            buf = ctypes.create_string_buffer(n)
            NativeRccl._check(runtime().ljs_comm_get_unique_id(buf), "ncclGetUniqueId")
            store.set(key, buf.raw)
            uid = buf.raw
        else:
            uid = store.get(key)
        out = _VP()
        NativeRccl._check(runtime().ljs_comm_init_rank(uid, self.world, self.rank, self.device, ctypes.byref(out)),
                          "ncclCommInitRank")
        return out.value

    def partition(self, groups: Tuple[Tuple[int, ...], ...]) -> Optional[int]:
        """Handle of this rank's communicator in a partition of the ranks into groups (None
        when this rank's group is a singleton).  Collective over every rank on first use."""
        if groups in self._parts:
            return self._parts[groups]
        mine = next((g for g in groups if self.rank in g), None)
        if mine is not None and sorted(mine) == list(range(self.world)):
            h = self._world_h
        else:
            color, key = -1, 0
            if mine is not None and len(mine) > 1:
                color = [g for g in groups if len(g) > 1].index(mine)
                key = sorted(mine).index(self.rank)
            out = _VP()
            NativeRccl._check(runtime().ljs_comm_split_rank(self._world_h, color, key, ctypes.byref(out)),
                              "ncclCommSplit")
            h = out.value if color >= 0 else None
        with self._mu:
            self._parts[groups] = h
        return h

    @staticmethod
    def supports(t: torch.Tensor) -> bool:
        from ..ops.hip import is_dense
        return t.is_cuda and t.dtype in _DT and is_dense(t)

    def _one(self, t):
        return (_VP * 1)(t.data_ptr())

    def _stream(self, t):
        return (_VP * 1)(torch.cuda.current_stream(t.device).cuda_stream)

    def all_reduce_(self, h: int, x: torch.Tensor) -> torch.Tensor:
        self._note(h, "all_reduce", x.numel() * x.element_size())
        NativeRccl._check(runtime().ljs_comm_all_reduce(h, self._one(x), self._one(x), x.numel(), _DT[x.dtype], 0,
                                                        self._stream(x)), "all_reduce")
        return x

    def all_gather(self, h: int, x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """out: [n * x.numel()] elements, rank-major."""
        self._note(h, "all_gather", x.numel() * x.element_size())
        NativeRccl._check(runtime().ljs_comm_all_gather(h, self._one(x), self._one(out), x.numel(), _DT[x.dtype],
                                                        self._stream(x)), "all_gather")
        return out

    def reduce_scatter(self, h: int, x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """x: n chunks of out.numel() elements (chunk r to rank r)."""
        self._note(h, "reduce_scatter", x.numel() * x.element_size())
        NativeRccl._check(runtime().ljs_comm_reduce_scatter(h, self._one(x), self._one(out), out.numel(),
                                                            _DT[x.dtype], 0, self._stream(x)), "reduce_scatter")
        return out

    def all_to_all(self, h: int, send: torch.Tensor, recv: torch.Tensor, n: int) -> torch.Tensor:
        self._note(h, "all_to_all", send.numel() * send.element_size())
        NativeRccl._check(runtime().ljs_comm_all_to_all(h, self._one(send), self._one(recv), send.numel() // n,
                                                        _DT[send.dtype], self._stream(send)), "all_to_all")
        return recv

    def _handles(self):
        hs = [self._world_h] if self._world_h else []
        with self._mu:
            parts = list(self._parts.values())
        for v in parts:
            if v and v not in hs:
                hs.append(v)
        return hs

    def _name(self, h) -> str:
        if h == self._world_h:
            return f"world ({self.world} ranks)"
        with self._mu:
            items = list(self._parts.items())
        for groups, v in items:
            if v == h:
                mine = next((g for g in groups if self.rank in g), ())
                return f"partition {list(map(list, groups))} (this rank's group {list(mine)})"
        return f"communicator {h:#x}"

    def query(self, h: Optional[int] = None) -> Dict[str, int]:
        """RCCL's own view of a communicator (default: the world one): ncclCommCount,
        ncclCommUserRank, ncclCommCuDevice."""
        h = self._world_h if h is None else h
        n, r, d = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
        NativeRccl._check(runtime().ljs_comm_query(h, ctypes.byref(n), ctypes.byref(r), ctypes.byref(d)),
                          "ncclCommCount")
        return {"nranks": n.value, "rank": r.value, "device": d.value}

    def partitions(self) -> Dict[Tuple[Tuple[int, ...], ...], Optional[int]]:
        with self._mu:
            return dict(self._parts)

    def check(self) -> None:
        """Failure detection: raise on the first asynchronous RCCL error of any of
        this rank's communicators (ncclCommGetAsyncError)."""
        for h in self._handles():
            rc = runtime().ljs_comm_async_error(h)
            if rc:
                raise RuntimeError(f"{self._name(h)}: {runtime().ljs_comm_error_string(rc).decode()}")

    def describe(self):
        """One line per communicator: its partition and the collectives issued on it (kinds,
        counts, bytes per call) - what a hang diagnosis prints (comm/watchdog.py)."""
        out = []
        for h in self._handles():
            with self._mu:
                ops = dict(self._log.get(h, {}))
            ops_s = ", ".join(f"{k} x{n} ({b / 1e6:.3g} MB/call)" for k, (n, b) in sorted(ops.items())) or "idle"
            out.append(f"{self._name(h)}: {ops_s}")
        return out

    def abort(self) -> None:
        """ncclCommAbort on every communicator (RCCL kernels waiting on a peer return)."""
        for h in self._handles():
            runtime().ljs_comm_abort(h)

    def close(self) -> None:
        """Destroy the partition communicators, then the world one (ncclCommDestroy)."""
        for h in self._handles()[::-1]:
            runtime().ljs_comm_destroy(h)
        with self._mu:
            self._parts.clear()
            self._world_h = None
            self._log.clear()

    def _note(self, h, kind: str, nbytes: int) -> None:
        with self._mu:
            ops = self._log.setdefault(h, {})
            n, b = ops.get(kind, (0, 0))
            ops[kind] = (n + 1, max(b, nbytes))
