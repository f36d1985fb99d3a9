"""Single-controller multi-GPU plumbing (comm/native.py, comm/backend.LocalComm) on the CPU
with a recording stand-in for the native RCCL runtime: communicator creation (ncclCommInitAll
over the visible GPUs, ncclCommSplit per device group with member-order keys), one grouped call
per device group with buffers in member (tile) order, and LocalComm's glue producing the same
results as its copy path."""
import ctypes

import pytest
import torch

from learning_jax_sharding_amd.comm import native
from learning_jax_sharding_amd.comm.backend import LocalComm


class FakeRuntime:
    """Records every ljs_comm_* call; handles are small integers."""

    def __init__(self):
        self.calls = []
        self._next = 100

    def _h(self):
        self._next += 1
        return self._next

    def ljs_comm_init(self, n, arr, out):
        self.calls.append(("init_all", tuple(arr[i] for i in range(n))))
        out._obj.value = self._h()
        return 0

    def ljs_comm_split(self, parent, colors, keys, n, out):
        world = len(self.calls[0][1])
        self.calls.append(("split", parent, tuple(colors[i] for i in range(world)), tuple(keys[i] for i in range(world))))
        out[0] = self._h()
        return 0

    def _coll(self, kind):
        def f(h, send, recv, count, dt, *rest):
            self.calls.append((kind, h, count, dt))
            return 0
        return f

    def __getattr__(self, name):
        kinds = {"ljs_comm_all_reduce": "all_reduce", "ljs_comm_all_gather": "all_gather",
                 "ljs_comm_reduce_scatter": "reduce_scatter", "ljs_comm_all_to_all": "all_to_all"}
        if name in kinds:
            return self._coll(kinds[name])
        raise AttributeError(name)


class _Dev:
    def __init__(self, i):
        self.type, self.index = "cuda", i


class _T:
    """Stand-in for a cuda tensor: only what NativeRccl reads."""

    def __init__(self, dev, n=8, dtype=torch.float32):
        self.device, self._n, self.dtype, self.shape = _Dev(dev), n, dtype, (n,)

    def __getitem__(self, i):  # a chunk of an [n, ...] all-to-all buffer
        return _T(self.device.index, 1, self.dtype)

    def data_ptr(self):
        return 4096 * (self.device.index + 1)

    def numel(self):
        return self._n


@pytest.fixture
def fake(monkeypatch):
    rt = FakeRuntime()
    monkeypatch.setattr(native, "runtime", lambda: rt)
    monkeypatch.setattr(native, "available", lambda: True)
    monkeypatch.setattr(native, "_streams", lambda ts: (ctypes.c_void_p * len(ts))(*[0] * len(ts)))
    monkeypatch.setattr(native, "_ptrs", lambda ts: (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts]))
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 4)
    return rt


def test_eligible_rules(monkeypatch):
    monkeypatch.setattr(native, "available", lambda: True)
    assert not native.eligible([torch.device("cpu"), torch.device("cpu")])
    assert not native.eligible([torch.device("cuda", 0)])                        # one member
    assert not native.eligible([torch.device("cuda", 0), torch.device("cuda", 0)])  # same GPU twice
    assert native.eligible([torch.device("cuda", 0), torch.device("cuda", 3)])
    monkeypatch.setenv("LJS_NATIVE_RCCL", "0")
    assert not native.eligible([torch.device("cuda", 0), torch.device("cuda", 3)])


def test_world_then_split_per_group_member_order(fake):
    nr = native.NativeRccl()
    h01 = nr.comm((0, 1))
    assert fake.calls[0] == ("init_all", (0, 1, 2, 3))            # the world: every visible GPU
    assert fake.calls[1][0] == "split"
    assert fake.calls[1][2] == (0, 0, -1, -1) and fake.calls[1][3] == (0, 1, 0, 0)
    # a group listed in tile order (2, 0): keys follow member order, not GPU order
    nr.comm((2, 0))
    assert fake.calls[-1][2] == (0, -1, 0, -1) and fake.calls[-1][3] == (1, 0, 0, 0)
    n = len(fake.calls)
    assert nr.comm((0, 1)) == h01 and len(fake.calls) == n         # cached


def test_one_grouped_call_per_group(fake, monkeypatch):
    real = torch.empty_like
    monkeypatch.setattr(torch, "empty_like", lambda t, *a, **k: _T(t.device.index, t._n) if isinstance(t, _T)
                        else real(t, *a, **k))
    nr = native.NativeRccl()
    ts = [_T(2), _T(0)]
    nr.all_reduce(ts)
    kinds = [c[0] for c in fake.calls]
    assert kinds.count("all_reduce") == 1                           # all members in ONE call
    assert fake.calls[-1][2] == 8 and fake.calls[-1][3] == native._DT[torch.float32]
    nr.all_to_all([_T(1, n=8), _T(3, n=8)])
    assert fake.calls[-1][0] == "all_to_all" and fake.calls[-1][2] == 1   # count per chunk (ts[0][0].numel())


class _FakeNative:
    """Native collectives computed with torch on CPU tensors, member order = list order."""

    def __init__(self):
        self.groups = []

    def all_gather(self, ts):
        self.groups.append(("ag", len(ts)))
        st = torch.stack(ts)
        return [st.clone() for _ in ts]

    def all_reduce(self, ts):
        self.groups.append(("ar", len(ts)))
        tot = sum(t.clone() for t in ts)
        for t in ts:
            t.copy_(tot)

    def reduce_scatter(self, ts):
        self.groups.append(("rs", len(ts)))
        tot = sum(t.clone() for t in ts)
        return [tot[i].clone() for i in range(len(ts))]

    def all_to_all(self, ts):
        self.groups.append(("a2a", len(ts)))
        n = len(ts)
        return [torch.stack([ts[j][i] for j in range(n)]) for i in range(n)]


@pytest.mark.parametrize("groups", [[(0, 1), (2, 3)], [(1, 0), (3, 2)], [(0, 2), (1, 3)], [(3, 1, 2, 0)]])
def test_localcomm_native_glue_matches_copy_path(monkeypatch, groups):
    g = torch.Generator().manual_seed(0)
    xs = {d: torch.randn(4, 6, generator=g) for d in range(4)}
    ref = LocalComm()
    want = {
        "ag": ref.all_gather(xs, groups, 1),
        "ar": ref.all_reduce(xs, groups),
        "a2a": ref.all_to_all(xs, groups, 0, 1),
    }
    rs_in = {d: torch.randn(len(groups[0]) * 2, 3, generator=torch.Generator().manual_seed(d)) for d in range(4)}
    want_rs = ref.reduce_scatter(rs_in, groups, 0)
    fake = _FakeNative()
    nat = LocalComm()
    monkeypatch.setattr(nat, "_rccl", lambda g_, xs_: fake)
    got_ag = nat.all_gather(xs, groups, 1)
    got_ar = nat.all_reduce(xs, groups)
    got_a2a = nat.all_to_all(xs, groups, 0, 1)
    got_rs = nat.reduce_scatter(rs_in, groups, 0)
    for d in range(4):
        torch.testing.assert_close(got_ag[d], want["ag"][d])
        torch.testing.assert_close(got_ar[d], want["ar"][d])
        torch.testing.assert_close(got_a2a[d], want["a2a"][d])
        torch.testing.assert_close(got_rs[d], want_rs[d])
    # one native call per device group and collective
    assert sorted(set(k for k, _ in fake.groups)) == ["a2a", "ag", "ar", "rs"]
    assert len(fake.groups) == 4 * len(groups)


class _Msg:
    """Tensor stand-in with the attributes DistComm's routing reads (a CPU box has no GPU tensors)."""
    def __init__(self, nbytes, dtype=torch.float32):
        self.is_cuda, self.dtype, self._n = True, dtype, nbytes // 4 if dtype == torch.float32 else nbytes // 2

    def numel(self):
        return self._n

    def element_size(self):
        return 4 if self.dtype == torch.float32 else 2


def test_p2p_route_graph_safe_only_when_group_built(monkeypatch):
    """The ipc peer-memory collectives are capturable (device-side barrier counter); DistComm
    reports a collective graph-safe only if it will take an already-built group that fits."""
    from learning_jax_sharding_amd.comm.backend import DistComm
    from learning_jax_sharding_amd.comm.p2p import P2PGroup
    monkeypatch.setenv("LJS_P2P", "1")
    c = object.__new__(DistComm)
    c.me, c._fake, c._native, c._p2p_groups = 1, False, None, {}
    groups = [(0, 1), (2, 3)]
    assert not c.graph_safe("all_reduce", _Msg(4096), groups)          # no group yet: torch path, cut
    grp = object.__new__(P2PGroup)
    grp.n, grp.cap, grp.oneshot_max = 2, 1 << 20, 256 << 10
    c._p2p_groups[(0, 1)] = grp
    assert c.graph_safe("all_reduce", _Msg(4096), groups)
    assert c.graph_safe("reduce_scatter", _Msg(4096), groups)
    assert not c.graph_safe("all_reduce", _Msg(2 << 20), groups)       # above LJS_P2P_MAX_KB
    assert not c.graph_safe("all_reduce", _Msg(4096), [(1, 2), (0, 3)])  # a different group
    assert not c.graph_safe("send", _Msg(4096), groups)
    monkeypatch.setenv("LJS_P2P", "0")
    assert not c.graph_safe("all_reduce", _Msg(4096), groups)


def test_p2p_auto_routing_follows_distinct_gpus(monkeypatch):
    """LJS_P2P unset ("auto"): small collectives take the peer-memory kernels exactly when every
    group member is a distinct GPU - an RCCL job's ranks, or a single controller's groups over
    several physical GPUs - and never for virtual devices of one GPU or a gloo / fake rehearsal."""
    import torch.distributed as dist
    from learning_jax_sharding_amd.comm import p2p
    from learning_jax_sharding_amd.comm.backend import DistComm, LocalComm
    from learning_jax_sharding_amd.comm.p2p import P2PGroup
    monkeypatch.delenv("LJS_P2P", raising=False)
    assert p2p.mode() == "auto" and p2p.wanted(True) and not p2p.wanted(False)
    monkeypatch.setenv("LJS_P2P", "1")
    assert p2p.wanted(False)
    monkeypatch.setenv("LJS_P2P", "0")
    assert not p2p.wanted(True)
    monkeypatch.delenv("LJS_P2P", raising=False)

    grp = object.__new__(P2PGroup)
    grp.n, grp.cap, grp.oneshot_max = 2, 1 << 20, 256 << 10
    groups = [(0, 1), (2, 3)]
    for backend, fake, want in [("nccl", False, True), ("gloo", False, False), ("nccl", True, False)]:
        c = object.__new__(DistComm)
        c.me, c._fake, c._native, c._p2p_groups = 1, fake, None, {(0, 1): grp}
        monkeypatch.setattr(dist, "get_backend", lambda *a, b=backend: b)
        assert c.graph_safe("all_reduce", _Msg(4096), groups) == want or fake, (backend, fake)
        assert c._p2p_ready("all_gather", _Msg(4096), groups) == want, (backend, fake)
        assert c.real_transfers() == want

    class _T:
        def __init__(self, idx):
            self.is_cuda, self.dtype, self.device = True, torch.float32, torch.device("cuda", idx)

        def numel(self):
            return 1024

        def element_size(self):
            return 4

    lc = LocalComm()
    built = []
    monkeypatch.setattr(p2p, "P2PGroup", lambda devs, cap: built.append(devs) or grp)
    assert lc._p2p((0, 1), {0: _T(0), 1: _T(0)}) is None               # virtual devices of one GPU
    assert lc._p2p((0, 1), {0: _T(0), 1: _T(1)}) is grp                # two GPUs
    assert len(built) == 1
    assert lc.real_transfers([torch.device("cuda", 0), torch.device("cuda", 1)])
    assert not lc.real_transfers([torch.device("cuda", 0), torch.device("cuda", 0)])


def test_qkv_prefetch_auto_only_for_real_transfers(monkeypatch):
    """The Q/K/V weight gather's side-stream prefetch (models/attention.py) is on by default
    exactly when the gather crosses GPUs (LJS_QKV_PREFETCH overrides)."""
    from learning_jax_sharding_amd.models import attention as A
    from learning_jax_sharding_amd.comm import backend as B

    class _W:
        def __init__(self, idxs):
            self.local = {i: type("t", (), {"device": torch.device("cuda", j)})() for i, j in enumerate(idxs)}

    class _Dist:
        kind = "dist"

        def __init__(self, real):
            self._real = real

        def real_transfers(self, devices=None):
            return self._real

    monkeypatch.setattr(A, "_QKV_PREFETCH", "auto")
    lc = B.LocalComm()
    monkeypatch.setattr(B, "get_comm", lambda: lc)
    assert not A.qkv_prefetch_wanted(_W([0, 0, 0, 0]))      # 4 virtual devices, one GPU
    assert A.qkv_prefetch_wanted(_W([0, 1, 2, 3]))          # single controller over 4 GPUs
    monkeypatch.setattr(B, "get_comm", lambda: _Dist(True))
    assert A.qkv_prefetch_wanted(_W([0]))                   # RCCL ranks
    monkeypatch.setattr(B, "get_comm", lambda: _Dist(False))
    assert not A.qkv_prefetch_wanted(_W([0]))               # fake / gloo rehearsal
    monkeypatch.setattr(A, "_QKV_PREFETCH", "1")
    assert A.qkv_prefetch_wanted(_W([0]))
    monkeypatch.setattr(A, "_QKV_PREFETCH", "0")
    monkeypatch.setattr(B, "get_comm", lambda: _Dist(True))
    assert not A.qkv_prefetch_wanted(_W([0]))
