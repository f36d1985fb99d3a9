"""Direct peer-memory collectives for small messages.

On an MI355X node every GPU pair has a dedicated xGMI link.  A ring collective (RCCL's bulk
algorithm) is per-link bound and pays 2(k-1) latency-bound steps; for the KB-to-MB messages
of the case6 plan a ONE-SHOT kernel that reads all k-1 peers at once uses every link and pays
one synchronisation.  Above ``oneshot_max`` the all-reduce is TWO-SHOT (peer-read
reduce-scatter into a result slot, barrier, peer-read all-gather), which moves 2(k-1)/k of
the message per GPU like a ring, but in two steps instead of 2(k-1).

Every member owns one staging allocation of fine-grained uncached device memory
(``ljs_p2p_alloc``): ``[flags 4 KiB | in: cap | res: cap]``.  In one-process-per-GPU runs the
allocations are exported by IPC handle (dmabuf, ``HSA_ENABLE_IPC_MODE_LEGACY=0``) and opened
by every other member; in single-controller runs they are peer-mapped.  Synchronisation:

* ``ipc`` mode: the flag barrier kernel of ``csrc/kernels/p2p.hip`` (system-scope stores into
  every member's flag array, device-side sequence counter, timeout -> error word, no hang);
* ``local`` mode: HIP events between the members' streams.

Routing (:func:`wanted`): by default every group whose members are distinct GPUs sends its
collectives of at most ``LJS_P2P_MAX_KB`` (default 1024) KiB per member through here - the
case6 2-D plan's K/V and head gathers and the out-projection all-to-all - and RCCL
keeps everything else; ``LJS_P2P=1`` forces the path on (virtual devices of one GPU too, for
tests), ``LJS_P2P=0`` off.  In ``ipc`` mode every collective is a staging
copy plus stream-ordered kernels whose barrier sequence comes from a device-side counter, so it
is captured into HIP graphs like a native RCCL call (``DistComm.graph_safe``) once the group
exists; the group itself (an IPC-handle exchange) is built by the eager warm-up call, never
inside a capture (``scripts/p2p_check.py`` replays a captured all-reduce + all-gather).
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Optional, Sequence

import torch

from ..ops import hip as _hip
from . import native as _native

__all__ = ["P2PGroup", "P2PUnavailable", "enabled", "wanted", "mode", "max_bytes"]


class P2PUnavailable(RuntimeError):
    """The group could not be built on some member (raised on EVERY member alike)."""

FLAG_BYTES = 4096          # 64 u32 arrival slots | word 64: sequence counter | word 65: error
_VP = ctypes.c_void_p
_DT = {torch.float32: 0, torch.bfloat16: 1}


def mode() -> str:
    """``LJS_P2P``: "1" every eligible small collective, "0" never, "auto" (default) only groups
    whose members are distinct physical GPUs - where the message crosses xGMI links."""
    v = os.environ.get("LJS_P2P", "auto").lower()
    return v if v in ("0", "1") else "auto"


def enabled() -> bool:
    """The peer-memory path may be taken at all (see :func:`wanted` for the per-group rule)."""
    return mode() != "0"


def wanted(distinct_gpus: bool) -> bool:
    """Whether a group's small collectives go through the peer-memory kernels: forced on / off
    by ``LJS_P2P``, else exactly when every member is a distinct GPU (virtual devices sharing one
    GPU keep the copy-based loopback path; ranks of a gloo rehearsal share GPUs or have none)."""
    m = mode()
    if m == "0":
        return False
    return m == "1" or bool(distinct_gpus)


def max_bytes() -> int:
    return int(float(os.environ.get("LJS_P2P_MAX_KB", "1024")) * 1024)


def _timeout_ms() -> int:
    return int(os.environ.get("LJS_P2P_TIMEOUT_MS", "10000"))


def _kern():
    L = _hip.lib()
    if not getattr(L, "_p2p_sigs", False):
        L.ljs_p2p_barrier.argtypes = [ctypes.POINTER(_VP), ctypes.c_int, ctypes.c_int, _VP, _VP, ctypes.c_long, _VP,
                                      _VP]
        L.ljs_p2p_reduce.argtypes = [ctypes.POINTER(_VP), ctypes.c_int, ctypes.c_long, _VP, ctypes.c_long,
                                     ctypes.c_int, _VP]
        L.ljs_p2p_gather.argtypes = [ctypes.POINTER(_VP), ctypes.c_int, ctypes.c_long, _VP, ctypes.c_long, _VP]
        L.ljs_p2p_copy.argtypes = [_VP, _VP, ctypes.c_long, _VP]
        for f in (L.ljs_p2p_barrier, L.ljs_p2p_reduce, L.ljs_p2p_gather, L.ljs_p2p_copy):
            f.restype = ctypes.c_int
        L._p2p_sigs = True
    return L


def _rt():
    L = _native.runtime()
    if not getattr(L, "_p2p_sigs", False):
        L.ljs_p2p_alloc.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(_VP), _VP]
        L.ljs_p2p_open.argtypes = [ctypes.c_int, _VP, ctypes.POINTER(_VP)]
        L.ljs_p2p_free.argtypes = [_VP]
        L.ljs_p2p_close.argtypes = [_VP]
        L.ljs_p2p_enable_peer.argtypes = [ctypes.c_int, ctypes.c_int]
        L.ljs_rt_capture_id.argtypes = [_VP, ctypes.POINTER(ctypes.c_ulonglong)]
        for f in (L.ljs_p2p_alloc, L.ljs_p2p_open, L.ljs_p2p_free, L.ljs_p2p_close, L.ljs_p2p_enable_peer,
                  L.ljs_rt_ipc_handle_size, L.ljs_rt_capture_id):
            f.restype = ctypes.c_int
        L._p2p_sigs = True
    return L


def _ck(rc, what):
    if rc:
        raise RuntimeError(f"p2p {what} failed with hipError {rc}")


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _capture_id(stream: int) -> int:
    """The capture sequence id of ``stream`` (0 when it is not capturing)."""
    cid = ctypes.c_ulonglong(0)
    rc = _rt().ljs_rt_capture_id(stream, ctypes.byref(cid))
    if rc < 0:
        raise RuntimeError(f"hipStreamGetCaptureInfo failed with hipError {-rc}")
    return int(cid.value)


class P2PGroup:
    """Staging buffers + collectives for one ordered group of members.

    ``devices[i]`` is member i's GPU.  ``rank`` is None in ``local`` mode (this process
    drives every member) or this process's member index in ``ipc`` mode, where construction
    is collective over ``pg`` (a torch.distributed group whose rank order is member order)."""

    def __init__(self, devices: Sequence[torch.device], capacity: int, rank: Optional[int] = None, pg=None):
        self.devices = [torch.device(d) for d in devices]
        self.n = len(self.devices)
        if not 1 <= self.n <= 8:
            raise ValueError("p2p groups hold 1..8 members")
        self.cap = (int(capacity) + 4095) // 4096 * 4096
        self.total = FLAG_BYTES + 2 * self.cap
        self.rank = rank
        self.mode = "local" if rank is None else "ipc"
        self.oneshot_max = int(os.environ.get("LJS_P2P_ONESHOT_KB", "256")) * 1024
        rt = _rt()
        self._own: List[int] = []     # allocations this process frees
        self._opened: List[int] = []  # peer mappings this process closes
        if self.mode == "local":
            self.base = []
            for d in self.devices:
                p = _VP()
                _ck(rt.ljs_p2p_alloc(d.index, self.total, ctypes.byref(p), None), "alloc")
                self.base.append(p.value)
                self._own.append(p.value)
            idx = sorted({d.index for d in self.devices})
            for a in idx:
                for b in idx:
                    _ck(rt.ljs_p2p_enable_peer(a, b), "enable_peer")
        else:
            # every step that can fail on one member is followed by an exchange of every member's
            # status, so the members agree: all of them raise P2PUnavailable (the caller routes
            # the group to RCCL) or none does - a lone failure never leaves peers waiting
            import torch.distributed as dist
            me = self.devices[rank]
            p = _VP()
            if rt.ljs_rt_ipc_handle_size() > 64:
                raise RuntimeError("unexpected IPC handle size")
            hbuf = (ctypes.c_uint8 * 64)()
            ok = rt.ljs_p2p_alloc(me.index, self.total, ctypes.byref(p), hbuf) == 0
            if ok:
                self._own.append(p.value)
            on_gpu = dist.get_backend(pg) == "nccl"
            mine = torch.tensor(list(hbuf) + [1 if ok else 0], dtype=torch.uint8, device=me if on_gpu else "cpu")
            allh = torch.empty(self.n * 65, dtype=torch.uint8, device=mine.device)
            dist.all_gather_into_tensor(allh, mine, group=pg)
            allh = allh.cpu().view(self.n, 65)
            if not bool(allh[:, 64].all()):
                self._release()
                raise P2PUnavailable(f"staging allocation failed on member(s) {allh[:, 64].eq(0).nonzero().flatten().tolist()}")
            self.base = []
            ok = True
            for r in range(self.n):
                if r == rank:
                    self.base.append(p.value)
                    continue
                h = (ctypes.c_uint8 * 64)(*allh[r].tolist()[:64])
                q = _VP()
                if rt.ljs_p2p_open(me.index, ctypes.cast(h, _VP), ctypes.byref(q)) != 0:
                    ok = False
                    break
                self.base.append(q.value)
                self._opened.append(q.value)
            st = torch.tensor([1 if ok else 0], dtype=torch.int32, device=mine.device)
            dist.all_reduce(st, op=dist.ReduceOp.MIN, group=pg)
            if int(st.item()) != 1:
                self._release()
                raise P2PUnavailable("opening a peer's IPC staging buffer failed")
        # per member: (stream, event, capture id) of the last collective's completion.  A group has
        # ONE staging buffer and ONE device-side barrier sequence, so two of its collectives must
        # never run concurrently: one issued on another stream (a side-stream weight prefetch next
        # to the compute stream's gathers, an async gradient bucket) first waits for the previous
        # one.  Every member issues its collectives in the same program order, so the executions -
        # and the barrier sequence numbers - line up on every member.
        self._last: Dict[int, tuple] = {}
        self.flags = (_VP * self.n)(*self.base)
        self.ins = (_VP * self.n)(*[b + FLAG_BYTES for b in self.base])
        self.res = (_VP * self.n)(*[b + FLAG_BYTES + self.cap for b in self.base])

    # ------------------------------------------------------------------ plumbing
    def _members(self) -> List[int]:
        return list(range(self.n)) if self.mode == "local" else [self.rank]

    def _enter(self):
        """Order this collective after the group's previous one when that ran on another stream:
        within the same capture, or both eager, through the previous one's completion event; an
        eager collective after one that was captured (and so runs inside graph replays) through
        the latest replay's completion event (spmd/graphs.py last_replay)."""
        from ..spmd.graphs import last_replay
        for m in self._members():
            s = torch.cuda.current_stream(self.devices[m])
            last = self._last.get(m)
            if last is None or last[0] == s.cuda_stream:
                continue
            cid = _capture_id(s.cuda_stream)
            if last[2] == cid:
                s.wait_event(last[1])
            elif cid == 0:
                ev = last_replay(self.devices[m].index)
                if ev is not None:
                    s.wait_event(ev)

    def _exit(self):
        for m in self._members():
            s = torch.cuda.current_stream(self.devices[m])
            ev = torch.cuda.Event()
            ev.record(s)
            self._last[m] = (s.cuda_stream, ev, _capture_id(s.cuda_stream))

    def _barrier(self):
        L = _kern()
        if self.mode == "ipc":
            b = self.base[self.rank]
            dev = self.devices[self.rank]
            _ck(L.ljs_p2p_barrier(self.flags, self.n, self.rank, b, b + 64 * 4, _timeout_ms(), b + 65 * 4,
                                  _stream(dev)), "barrier")
            return
        evs = []
        for d in self.devices:
            e = torch.cuda.Event()
            e.record(torch.cuda.current_stream(d))
            evs.append(e)
        for d in self.devices:
            s = torch.cuda.current_stream(d)
            for e in evs:
                s.wait_event(e)

    def _stage(self, xs: Dict[int, torch.Tensor], nbytes: int):
        L = _kern()
        for m in self._members():
            x = xs[m]
            with torch.cuda.device(self.devices[m]):
                _ck(L.ljs_p2p_copy(self.ins[m], x.data_ptr(), nbytes, _stream(self.devices[m])), "copy")

    def fits(self, nbytes: int, chunked: bool = False) -> bool:
        """Whether a message of ``nbytes`` per member can go through this group (``chunked``:
        it is split into n equal 16-byte-aligned chunks, as reduce-scatter / all-to-all /
        two-shot all-reduce do)."""
        if not 0 < nbytes <= self.cap or nbytes % 16:
            return False
        if chunked or nbytes > self.oneshot_max:
            return nbytes % (16 * self.n) == 0
        return True

    def check_error(self):
        """Raise if a barrier of this member timed out (lost or wedged peer)."""
        for m in self._members():
            with torch.cuda.device(self.devices[m]):
                torch.cuda.current_stream(self.devices[m]).synchronize()
            word = torch.empty(1, dtype=torch.int32, device=self.devices[m])
            _ck(_kern().ljs_p2p_copy(word.data_ptr(), self.base[m] + 65 * 4, 4, _stream(self.devices[m])), "copy")
            if int(word.item()) != 0:
                raise RuntimeError(f"p2p barrier timed out on member {m} (a peer never arrived)")

    # ------------------------------------------------------------------ collectives
    def all_reduce(self, xs: Dict[int, torch.Tensor], out: Optional[Dict[int, torch.Tensor]] = None):
        """Sum of the members' contiguous tensors (f32 / bf16, f32 accumulation in member
        order: every member's result is bitwise identical).  ``xs``/``out`` keyed by member."""
        x0 = xs[self._members()[0]]
        nbytes = x0.numel() * x0.element_size()
        dt = _DT[x0.dtype]
        out = out if out is not None else {m: torch.empty_like(xs[m]) for m in self._members()}
        L = _kern()
        self._enter()
        self._stage(xs, nbytes)
        self._barrier()
        if nbytes <= self.oneshot_max:
            for m in self._members():
                with torch.cuda.device(self.devices[m]):
                    _ck(L.ljs_p2p_reduce(self.ins, self.n, 0, out[m].data_ptr(), nbytes, dt,
                                         _stream(self.devices[m])), "reduce")
        else:
            chunk = nbytes // self.n
            for m in self._members():
                with torch.cuda.device(self.devices[m]):
                    _ck(L.ljs_p2p_reduce(self.ins, self.n, m * chunk, self.res[m], chunk, dt,
                                         _stream(self.devices[m])), "reduce")
            self._barrier()
            for m in self._members():
                with torch.cuda.device(self.devices[m]):
                    _ck(L.ljs_p2p_gather(self.res, self.n, 0, out[m].data_ptr(), chunk, _stream(self.devices[m])),
                        "gather")
        self._barrier()
        self._exit()
        return out

    def all_gather(self, xs: Dict[int, torch.Tensor]):
        """Per member a [n, *shape] tensor of every member's block, member-major."""
        x0 = xs[self._members()[0]]
        nbytes = x0.numel() * x0.element_size()
        out = {m: torch.empty((self.n,) + tuple(xs[m].shape), dtype=xs[m].dtype, device=xs[m].device)
               for m in self._members()}
        L = _kern()
        self._enter()
        self._stage(xs, nbytes)
        self._barrier()
        for m in self._members():
            with torch.cuda.device(self.devices[m]):
                _ck(L.ljs_p2p_gather(self.ins, self.n, 0, out[m].data_ptr(), nbytes, _stream(self.devices[m])),
                    "gather")
        self._barrier()
        self._exit()
        return out

    def reduce_scatter(self, xs: Dict[int, torch.Tensor]):
        """xs[m] is [n, *chunk] (chunk r destined to member r): each member's summed chunk."""
        x0 = xs[self._members()[0]]
        nbytes = x0.numel() * x0.element_size()
        chunk = nbytes // self.n
        out = {m: torch.empty(tuple(xs[m].shape[1:]), dtype=xs[m].dtype, device=xs[m].device)
               for m in self._members()}
        L = _kern()
        self._enter()
        self._stage(xs, nbytes)
        self._barrier()
        for m in self._members():
            with torch.cuda.device(self.devices[m]):
                _ck(L.ljs_p2p_reduce(self.ins, self.n, m * chunk, out[m].data_ptr(), chunk, _DT[x0.dtype],
                                     _stream(self.devices[m])), "reduce")
        self._barrier()
        self._exit()
        return out

    def all_to_all(self, xs: Dict[int, torch.Tensor]):
        """xs[m] is [n, *chunk]; chunk r of member i lands as chunk i of member r."""
        x0 = xs[self._members()[0]]
        nbytes = x0.numel() * x0.element_size()
        chunk = nbytes // self.n
        out = {m: torch.empty_like(xs[m]) for m in self._members()}
        L = _kern()
        self._enter()
        self._stage(xs, nbytes)
        self._barrier()
        for m in self._members():
            with torch.cuda.device(self.devices[m]):
                _ck(L.ljs_p2p_gather(self.ins, self.n, m * chunk, out[m].data_ptr(), chunk, _stream(self.devices[m])),
                    "gather")
        self._barrier()
        self._exit()
        return out

    def _release(self):
        rt = _rt()
        for p in self._opened:
            rt.ljs_p2p_close(p)
        for p in self._own:
            rt.ljs_p2p_free(p)
        self._opened, self._own = [], []

    def close(self):
        for m in self._members():
            torch.cuda.current_stream(self.devices[m]).synchronize()
        self._release()
