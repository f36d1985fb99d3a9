"""HIP-graph capture cut at collectives ("segmented graphs").

``jit(..., capture=True)`` replays a whole step as HIP graphs instead of re-running Python.
In one-process-per-GPU runs the step contains RCCL collectives; rather than relying on
collective capture inside graphs, the capture is CUT at every cross-process collective:

    graph 0 | collective 0 (eager) | graph 1 | collective 1 (eager) | ... | graph n

All segments share one graph memory pool, so tensors produced by one segment keep their
addresses for the next; a collective's inputs are such static tensors and its outputs are
allocated once at capture time.  On replay each graph is replayed and each collective
re-issued on the same stream order, its fresh result copied into the static output.

A collective may also be issued ASYNCHRONOUSLY (data-parallel gradient buckets): it then
runs on a side comm stream, concurrent with the following graph segments, and the
consumer joins it with :func:`join` (an event wait, also replayed in order).

Collectives of the native RCCL rank communicators (``comm/native.py`` ``RankRccl``) are plain
RCCL calls on the current stream and are NOT cut points: they are captured with the kernels
(asynchronous ones forked onto a side stream inside the capture), so a data-parallel train step
replays as a single graph.  The cut path remains for torch process-group collectives (gloo, or
``LJS_NATIVE_RCCL=0``).
"""
from __future__ import annotations

import os
import sys
import warnings
from typing import Any, Callable, Dict, List, Optional

import torch

__all__ = ["SegmentedGraph", "MultiDeviceGraph", "current", "run_collective", "join"]

# process-wide (one capture at a time)
_ACTIVE: List[Optional["SegmentedGraph"]] = [None]


# callables run before a capture segment ends: work deferred inside the segment that must be in
# it (the optimizer's pending count increments, ops/hip._flush_step_incs) is launched there
BEFORE_CUT: List[Callable[[], None]] = []


def _before_cut() -> None:
    for fn in BEFORE_CUT:
        fn()


# callables run when a whole capture ends (state that must not leak into later calls)
AFTER_CAPTURE: List[Callable[[], None]] = []


def current() -> Optional["SegmentedGraph"]:
    return _ACTIVE[0]


def _copy_into(dst, src):
    if isinstance(dst, dict):
        for k, v in dst.items():
            _copy_into(v, src[k])
    elif isinstance(dst, (list, tuple)):
        for a, b in zip(dst, src):
            _copy_into(a, b)
    elif isinstance(dst, torch.Tensor):
        # (detached: a static output may be the view an autograd Function returned at capture, e.g.
        # a 2-D layout's gathered K / V -- its refresh is data movement, not a differentiable op)
        dst.detach().copy_(src.detach() if isinstance(src, torch.Tensor) else src)


class SegmentedGraph:
    def __init__(self):
        self.pool = torch.cuda.graph_pool_handle()
        self.items: List[tuple] = []
        self._g: Optional[torch.cuda.CUDAGraph] = None
        self._origin: Optional[torch.cuda.Stream] = None   # the stream every segment begins / ends on
        self.comm_stream: Optional[torch.cuda.Stream] = None
        self.n_collectives = 0

    # ------------------------------------------------------------------ capture
    def _begin(self):
        self._g = torch.cuda.CUDAGraph()
        cur = torch.cuda.current_stream()
        # HIP ends a capture only on the thread that began it, so value_and_grad runs the
        # backward single-threaded while a segmented capture is active (cuts happen inside it)
        with torch.cuda.stream(self._origin):
            self._g.capture_begin(pool=self.pool, capture_error_mode="relaxed")
        if cur != self._origin:
            # a cut made on a forked stream: that stream joins the new segment again
            cur.wait_stream(self._origin)

    def _cut(self):
        _before_cut()
        cur = torch.cuda.current_stream()
        if cur != self._origin:
            # a collective issued on a stream forked inside the capture (a side-stream gather):
            # the fork joins the segment's own stream, which ends the capture (a capture must end
            # on the stream it began on, with every fork joined)
            self._origin.wait_stream(cur)
        with warnings.catch_warnings():
            # two adjacent cut points leave an empty segment: harmless, replays as a no-op
            warnings.filterwarnings("ignore", message="The CUDA Graph is empty")
            with torch.cuda.stream(self._origin):
                self._g.capture_end()
        self.items.append(("graph", self._g))
        self._g = None

    def capture(self, fn: Callable[[], Any]):
        """Run ``fn`` once under segmented capture (on a side stream, as HIP graph capture
        requires); returns its outputs (static tensors)."""
        torch.cuda.synchronize()
        stream = torch.cuda.Stream()
        stream.wait_stream(torch.cuda.current_stream())
        prev = current()
        _ACTIVE[0] = self
        self._origin = stream
        try:
            with torch.cuda.stream(stream):
                self._begin()
                try:
                    out = fn()
                finally:
                    if self._g is not None:
                        self._cut()
                    for f in AFTER_CAPTURE:
                        f()
        finally:
            _ACTIVE[0] = prev
        torch.cuda.current_stream().wait_stream(stream)
        torch.cuda.synchronize()
        return out

    def collective(self, fn: Callable[[], Any], async_: bool = False):
        """Inside capture: cut the graph, run ``fn`` eagerly, record it for replay."""
        self._cut()
        self.n_collectives += 1
        if async_:
            if self.comm_stream is None:
                self.comm_stream = torch.cuda.Stream()
            cur = torch.cuda.current_stream()
            self.comm_stream.wait_stream(cur)
            with torch.cuda.stream(self.comm_stream):
                out = fn()
            ev = torch.cuda.Event()
            ev.record(self.comm_stream)
            self.items.append(("async", fn, out, ev))
            handle = ev
        else:
            out = fn()
            self.items.append(("sync", fn, out))
            handle = None
        self._begin()
        return out, handle

    def side_stream(self) -> torch.cuda.Stream:
        """Stream for collectives forked inside the capture (joined before the capture ends)."""
        if self.comm_stream is None:
            self.comm_stream = torch.cuda.Stream()
        return self.comm_stream

    def join(self, ev: torch.cuda.Event):
        self._cut()
        torch.cuda.current_stream().wait_event(ev)
        self.items.append(("join", ev))
        self._begin()

    # ------------------------------------------------------------------ replay
    def replay(self):
        cur = torch.cuda.current_stream()
        try:
            self._replay(cur)
        finally:
            _note_replay({torch.cuda.current_device(): cur})

    def _replay(self, cur):
        for it in self.items:
            kind = it[0]
            if kind == "graph":
                it[1].replay()
            elif kind == "sync":
                _copy_into(it[2], it[1]())
            elif kind == "async":
                _, fn, out, ev = it
                self.comm_stream.wait_stream(cur)
                with torch.cuda.stream(self.comm_stream):
                    _copy_into(out, fn())
                ev.record(self.comm_stream)
            elif kind == "join":
                cur.wait_event(it[1])


class _Fork:
    """Join handle of a collective forked onto a side stream INSIDE a capture (no cut)."""
    __slots__ = ("ev",)

    def __init__(self, ev):
        self.ev = ev


def run_collective(fn: Callable[[], Any], async_: bool = False, capturable: bool = False, what: str = ""):
    """Issue a cross-process collective: directly (eager), as a cut point of the active
    segmented capture, or - when ``capturable`` (native RCCL on the current stream) - as part
    of the capture itself, forked onto a side stream when ``async_`` so it overlaps the rest of
    the captured step.  Returns (outputs, join handle or None)."""
    seg = current()
    if seg is not None and capturable:
        if not async_:
            return fn(), None
        cur = torch.cuda.current_stream()
        cs = seg.side_stream()
        cs.wait_stream(cur)
        with torch.cuda.stream(cs):
            out = fn()
        ev = torch.cuda.Event()
        ev.record(cs)
        return out, _Fork(ev)
    if seg is None:
        if async_ and torch.cuda.is_available():
            cs = _side_stream()
            cs.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(cs):
                out = fn()
            ev = torch.cuda.Event()
            ev.record(cs)
            return out, ev
        return fn(), None
    if _CUT_TRACE:
        # diagnostics (LJS_GRAPH_CUT_TRACE=1): where a capture is cut, i.e. which collective took a
        # path that cannot be captured
        import traceback
        fr = [f for f in traceback.extract_stack(limit=8)[:-1] if "spmd/graphs.py" not in f.filename]
        print(f"[ljs graph cut] {what or 'collective'} at " + " <- ".join(f"{f.filename.rsplit('/', 2)[-1]}:{f.lineno}"
                                                                           for f in reversed(fr[-4:])),
              file=sys.stderr, flush=True)
    return seg.collective(fn, async_)


_CUT_TRACE = os.environ.get("LJS_GRAPH_CUT_TRACE", "0") == "1"


def forks_ok() -> bool:
    """Whether work may be forked onto a side stream now (a prefetched gather, a ring hop).
    Inside a segmented capture whose collectives are cut points (torch process-group
    collectives: gloo, or RCCL without the native rank communicators) a fork still open at a cut
    would leave the segment unjoined, so the forking sites run on the current stream there -- the
    cut collectives run eagerly and in order anyway, there is nothing to overlap them with."""
    seg = current()
    if seg is None or isinstance(seg, MultiDeviceGraph):
        return True
    from ..comm.backend import get_comm
    return not get_comm().cuts_capture()


def join(handle) -> None:
    """Make the current stream wait for an asynchronous collective."""
    if handle is None:
        return
    if isinstance(handle, _Fork):
        torch.cuda.current_stream().wait_event(handle.ev)
        return
    seg = current()
    if seg is not None:
        seg.join(handle)
    else:
        torch.cuda.current_stream().wait_event(handle)


# per device: an event recorded on the replay stream after the latest graph replay.  Work issued
# eagerly on ANOTHER stream that shares state with the graph's collectives (the p2p groups' one
# staging buffer and barrier sequence, comm/p2p.py _enter) waits on it: an event recorded inside
# a capture cannot be waited on outside it.
_LAST_REPLAY: Dict[int, Any] = {}
# record the completion event after every replay instead of lazily (tests)
_EAGER_REPLAY_EVENT = False


def _note_replay(streams: Dict[int, Any]) -> None:
    """Remember the stream each device's latest replay ran on.  The completion event is recorded
    only when someone asks for it (:func:`last_replay`, the P2P collectives' ordering): an event
    recorded on that stream later still follows the replay.  Recorded after every replay (the
    round-4 form) it put a marker packet between consecutive graph launches."""
    if _EAGER_REPLAY_EVENT:
        for d, s in streams.items():
            with torch.cuda.device(d):
                ev = torch.cuda.Event()
                ev.record(s)
            _LAST_REPLAY[d] = ev
        return
    for d, s in streams.items():
        _LAST_REPLAY[d] = s


def last_replay(device: int):
    """An event that completes after the latest graph replay on ``device`` (or None)."""
    e = _LAST_REPLAY.get(device)
    if e is None or isinstance(e, torch.cuda.Event):
        return e
    with torch.cuda.device(device):
        ev = torch.cuda.Event()
        ev.record(e)
    _LAST_REPLAY[device] = ev
    return ev


_SIDE: Dict[int, torch.cuda.Stream] = {}


def _side_stream() -> torch.cuda.Stream:
    d = torch.cuda.current_device()
    s = _SIDE.get(d)
    if s is None:
        s = _SIDE[d] = torch.cuda.Stream()
    return s


# ============================================================================ single controller, N GPUs
class _TorchMD:
    """The torch / HIP calls of a multi-device capture (a test double replaces them)."""

    def synchronize(self, devs):
        for d in devs:
            torch.cuda.synchronize(d)

    def new_stream(self, d):
        return torch.cuda.Stream(device=d)

    def current_stream(self, d):
        return torch.cuda.current_stream(d)

    def new_graph(self):
        return torch.cuda.CUDAGraph()

    def pool(self):
        return torch.cuda.graph_pool_handle()

    def device(self, d):
        return torch.cuda.device(d)

    def stream(self, s):
        return torch.cuda.stream(s)

    def event(self):
        return torch.cuda.Event()

    def begin_pool(self, d, pool):
        # every allocation on device d until end_pool comes from the graph's private pool there
        # (the capturing device's pool is routed by capture_begin itself)
        torch._C._cuda_beginAllocateToPool(d, pool)

    def end_pool(self, d, pool):
        torch._C._cuda_endAllocateToPool(d, pool)

    def release_pool(self, d, pool):
        torch._C._cuda_releasePool(d, pool)


class MultiDeviceGraph:
    """ONE hipGraph of a single-controller step over several physical GPUs (the reference's own
    execution model: one process, N devices, ``case6_attention.py:4-5,219-220``).

    The capture begins on the first device's capture stream; every other device's capture stream
    joins it through an event wait (a fork inside the capture), so the work the step issues on
    each device's current stream - kernels, the grouped single-controller RCCL calls of
    ``comm/native.py``, the peer-memory collectives' cross-device event waits - becomes nodes of
    the same graph, with the cross-device orders as graph edges.  Each device's allocations go
    to a private pool for the graph's lifetime (the capturing device's through ``capture_begin``,
    the others' through the allocator's pool routing).  The other devices join back before the
    capture ends.  Replay is one graph launch."""

    def __init__(self, devices, backend=None):
        self.devices = sorted(set(int(d) for d in devices))
        self.be = backend or _TorchMD()
        self.graph = None
        self.pools: Dict[int, Any] = {}
        self.items: List[tuple] = []
        self.n_collectives = 0

    def capture(self, fn: Callable[[], Any]):
        import contextlib
        be, devs = self.be, self.devices
        d0, others = devs[0], devs[1:]
        be.synchronize(devs)
        streams = {d: be.new_stream(d) for d in devs}
        for d in devs:
            streams[d].wait_stream(be.current_stream(d))
        g = be.new_graph()
        prev = current()
        began = []
        with contextlib.ExitStack() as cx:
            for d in devs:
                cx.enter_context(be.stream(streams[d]))   # each device's current stream: its capture stream
            with be.device(d0):
                g.capture_begin(pool=be.pool(), capture_error_mode="relaxed")
            try:
                fork = be.event()
                with be.device(d0):
                    fork.record(streams[d0])
                for d in others:
                    with be.device(d):
                        streams[d].wait_event(fork)       # joins the capture
                        pool = be.pool()
                        be.begin_pool(d, pool)
                        self.pools[d] = pool
                        began.append(d)
                _ACTIVE[0] = self    # (single-threaded backward; collectives are graph nodes, no cuts)
                out = fn()
                for d in others:
                    with be.device(d):
                        ev = be.event()
                        ev.record(streams[d])
                    streams[d0].wait_event(ev)            # join back before the capture ends
            finally:
                _ACTIVE[0] = prev
                for d in began:
                    be.end_pool(d, self.pools[d])
                with be.device(d0):
                    g.capture_end()
        for d in devs:
            be.current_stream(d).wait_stream(streams[d])
        be.synchronize(devs)
        self.graph = g
        self.items = [("graph", g)]
        return out

    # the SegmentedGraph interface of run_collective / join: nothing is cut here - a collective is
    # issued on the current (capturing) streams and becomes part of the graph
    def collective(self, fn: Callable[[], Any], async_: bool = False):
        self.n_collectives += 1
        return fn(), None

    def side_stream(self):
        return _side_stream()

    def join(self, ev):
        torch.cuda.current_stream().wait_event(ev)

    def replay(self):
        """One graph launch on d0's current stream, ordered against every device's current stream
        on both sides: the graph's branches on device d read inputs that ``Jitted._replay`` copied
        on d's own current stream (so d0's stream waits for each of them before the launch), and
        later work on d - including the next replay's input copies into the buffers this one is
        still reading - waits for the whole graph (each device's stream waits on d0's after it)."""
        be, devs = self.be, self.devices
        d0, others = devs[0], devs[1:]
        s0 = be.current_stream(d0)
        for d in others:
            with be.device(d):
                ev = be.event()
                ev.record(be.current_stream(d))
            s0.wait_event(ev)
        with be.device(d0):
            self.graph.replay()
            done = be.event()
            done.record(s0)
        for d in others:
            be.current_stream(d).wait_event(done)
        if isinstance(be, _TorchMD):
            _note_replay({d: be.current_stream(d) for d in devs})

    def release(self):
        """Return the other devices' pools (the graph keeps its own device's)."""
        for d, pool in self.pools.items():
            self.be.release_pool(d, pool)
        self.pools = {}

    def __del__(self):
        try:
            if self.pools and self.graph is not None:
                self.graph = None
                self.release()
        except Exception:
            pass
