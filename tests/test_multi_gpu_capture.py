"""Single-controller multi-GPU capture (spmd/graphs.py MultiDeviceGraph) with a recording test
double for the torch / HIP calls (no GPU here): one graph per step, every device's capture
stream forked from the first device's inside the capture, each device's allocations in a private
pool, the step's collectives issued on the capturing streams (graph nodes, no cuts), the branches
joined back before the capture ends; replay is one graph launch."""
import contextlib

from learning_jax_sharding_amd.spmd import graphs


class _Ev:
    def __init__(self, log, n):
        self.log, self.n, self.stream = log, n, None

    def record(self, s):
        self.stream = s
        self.log.append(("record", self.n, s.dev))


class _Stream:
    def __init__(self, log, dev, name):
        self.log, self.dev, self.name = log, dev, name

    def wait_stream(self, other):
        self.log.append(("wait_stream", self.dev, other.dev))

    def wait_event(self, ev):
        self.log.append(("wait_event", self.dev, ev.n, ev.stream.dev))


class _Graph:
    def __init__(self, log):
        self.log = log

    def capture_begin(self, pool=None, capture_error_mode="global"):
        self.log.append(("capture_begin", self.log_dev[0], capture_error_mode))

    def capture_end(self):
        self.log.append(("capture_end", self.log_dev[0]))

    def replay(self):
        self.log.append(("replay",))


class _Backend:
    def __init__(self):
        self.log = []
        self.cur = {}
        self.dev = [None]
        self.n_ev = 0
        self.n_pool = 0

    def synchronize(self, devs):
        self.log.append(("sync", tuple(devs)))

    def new_stream(self, d):
        return _Stream(self.log, d, f"cap{d}")

    def current_stream(self, d):
        return self.cur.get(d) or _Stream(self.log, d, f"default{d}")

    def new_graph(self):
        g = _Graph(self.log)
        g.log_dev = self.dev
        return g

    def pool(self):
        self.n_pool += 1
        return (self.n_pool, 0)

    @contextlib.contextmanager
    def device(self, d):
        prev = self.dev[0]
        self.dev[0] = d
        try:
            yield
        finally:
            self.dev[0] = prev

    @contextlib.contextmanager
    def stream(self, s):
        prev = self.cur.get(s.dev)
        self.cur[s.dev] = s
        try:
            yield
        finally:
            if prev is None:
                self.cur.pop(s.dev)
            else:
                self.cur[s.dev] = prev

    def event(self):
        self.n_ev += 1
        return _Ev(self.log, self.n_ev)

    def begin_pool(self, d, pool):
        self.log.append(("begin_pool", d, pool))

    def end_pool(self, d, pool):
        self.log.append(("end_pool", d, pool))

    def release_pool(self, d, pool):
        self.log.append(("release_pool", d, pool))


def test_multi_device_graph_capture_structure():
    be = _Backend()
    g = graphs.MultiDeviceGraph([2, 0, 1, 3], backend=be)
    issued = []

    def step():
        # the step sees every device's CAPTURE stream as current, and no cut-point capture
        assert graphs.current() is g
        for d in range(4):
            assert be.current_stream(d).name == f"cap{d}"
        # a collective over the devices (issued on the current streams: a node of the graph)
        out, h = graphs.run_collective(lambda: issued.append("all_reduce") or "ok", capturable=False)
        assert out == "ok" and h is None
        return "out"

    assert g.capture(step) == "out"
    assert issued == ["all_reduce"] and g.n_collectives == 1
    log = be.log
    kinds = [e[0] for e in log]
    # exactly one capture, begun and ended on the first device
    assert kinds.count("capture_begin") == 1 and kinds.count("capture_end") == 1
    assert ("capture_begin", 0, "relaxed") in log and ("capture_end", 0) in log
    b, e = kinds.index("capture_begin"), kinds.index("capture_end")
    # devices 1..3 fork from device 0's capture stream inside the capture, with private pools
    fork = next(x for x in log[b:e] if x[0] == "record")
    for d in (1, 2, 3):
        assert ("wait_event", d, fork[1], 0) in log[b:e]
        assert any(x[0] == "begin_pool" and x[1] == d for x in log[b:e])
        assert any(x[0] == "end_pool" and x[1] == d for x in log)
    # ... and join back into device 0 before the capture ends
    joins = [x for x in log[b:e] if x[0] == "wait_event" and x[1] == 0]
    assert sorted(x[3] for x in joins) == [1, 2, 3]
    assert graphs.current() is None
    n0 = len(log)
    g.replay()
    rl = log[n0:]
    assert [x[0] for x in rl].count("replay") == 1
    r = [x[0] for x in rl].index("replay")
    # device 0's stream waits for every other device's current stream before the launch ...
    assert sorted(x[3] for x in rl[:r] if x[0] == "wait_event" and x[1] == 0) == [1, 2, 3]
    # ... and every other device's current stream waits for the launch after it
    assert sorted(x[1] for x in rl[r:] if x[0] == "wait_event" and x[3] == 0) == [1, 2, 3]
    g.release()
    assert sorted(x[1] for x in log if x[0] == "release_pool") == [1, 2, 3]


def test_multi_device_graph_failure_releases_pools():
    be = _Backend()
    g = graphs.MultiDeviceGraph([0, 1], backend=be)

    def bad():
        raise RuntimeError("operation not permitted when stream is capturing")

    try:
        g.capture(bad)
        raise AssertionError("expected the capture to fail")
    except RuntimeError:
        pass
    kinds = [x[0] for x in be.log]
    assert kinds.count("capture_end") == 1 and ("end_pool", 1, g.pools[1]) in be.log
    assert graphs.current() is None


def test_jit_uses_multi_device_capture_when_steps_span_gpus(monkeypatch):
    """A captured jit whose devices span several GPUs captures through MultiDeviceGraph (no
    longer eager); a runtime that refuses falls back to eager for that signature."""
    import torch
    from learning_jax_sharding_amd.spmd import api
    seen = []

    class _MD:
        def __init__(self, devs):
            seen.append(tuple(devs))
            self.items = []

        def capture(self, fn):
            return fn()

        def replay(self):
            seen.append("replay")

        def release(self):
            pass

    monkeypatch.setattr(api, "_MULTI_GPU_CAPTURE", True)
    monkeypatch.setattr(api, "_spans_gpus", lambda: True)
    monkeypatch.setattr(api, "_gpu_indices", lambda: [0, 1])
    monkeypatch.setattr(graphs, "MultiDeviceGraph", _MD)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a: None)
    calls = []

    def f(x):
        calls.append(1)
        return x

    j = api.jit(f, capture=True)
    j(1.0)                 # warm-up call (eager)
    j(1.0)                 # captured through the multi-device graph
    assert seen and seen[0] == (0, 1)


def test_forks_ok_follows_capture_cuts(monkeypatch):
    """Side-stream forks are skipped only inside a segmented capture whose collectives cut it
    (torch process-group collectives); native RCCL / rehearsal collectives are captured, and a
    single-controller multi-device capture never cuts."""
    from learning_jax_sharding_amd.comm import backend

    class _Comm:
        def __init__(self, cuts):
            self.cuts = cuts

        def cuts_capture(self):
            return self.cuts

    assert graphs.forks_ok()                       # no capture
    prev = graphs._ACTIVE[0]
    try:
        graphs._ACTIVE[0] = graphs.SegmentedGraph.__new__(graphs.SegmentedGraph)
        monkeypatch.setattr(backend, "get_comm", lambda: _Comm(True))
        assert not graphs.forks_ok()
        monkeypatch.setattr(backend, "get_comm", lambda: _Comm(False))
        assert graphs.forks_ok()
        graphs._ACTIVE[0] = graphs.MultiDeviceGraph([0, 1], backend=object())
        monkeypatch.setattr(backend, "get_comm", lambda: _Comm(True))
        assert graphs.forks_ok()
    finally:
        graphs._ACTIVE[0] = prev
