"""Peer-memory (P2P) collective fallbacks are recorded, not fatal (verdict r5 item 3): a group
whose build fails stays on RCCL with the reason, and a barrier timeout detected at run time moves
every later collective of the job to RCCL -- both visible in ``DistComm.comm_detail()``.

Mock-level: a DistComm built without a process group (``__new__``), its torch.distributed calls
replaced, and P2PGroup replaced by doubles; the path choice and the records are what is tested."""
import pytest
import torch

from learning_jax_sharding_amd.comm import backend as B
from learning_jax_sharding_amd.comm import p2p


class _Dist:
    """The torch.distributed surface DistComm touches here."""
    ReduceOp = torch.distributed.ReduceOp

    def __init__(self, peer_failed=False):
        self.peer_failed = peer_failed

    def get_backend(self, *_):
        return "nccl"

    def get_world_size(self):
        return 2

    def all_reduce(self, t, op=None, group=None):
        if self.peer_failed:
            t.fill_(1)


class _Grp:
    oneshot_max = 1 << 18

    def __init__(self, *a, timed_out=False, **k):
        self.timed_out, self.closed = timed_out, False

    def fits(self, nbytes, chunked=False):
        return True

    def check_error(self):
        if self.timed_out:
            raise RuntimeError("p2p barrier timed out on member 0 (a peer never arrived)")

    def close(self):
        self.closed = True


def _comm(monkeypatch, dist):
    monkeypatch.setattr(B, "dist", dist)
    c = B.DistComm.__new__(B.DistComm)
    c.me, c._p2p_groups, c._fake, c._native = 0, {}, False, None
    c.routes, c.p2p_fallbacks, c._p2p_off = {}, [], None
    monkeypatch.setattr(c, "_distinct_gpus", lambda: True)
    return c


class _X:
    """A CUDA-looking f32 tensor (routing checks only look at these attributes)."""
    is_cuda, dtype, device = True, torch.float32, torch.device("cuda", 0)

    def numel(self):
        return 256

    def element_size(self):
        return 4


def test_build_failure_stays_on_rccl_with_reason(monkeypatch):
    c = _comm(monkeypatch, _Dist())
    monkeypatch.setenv("LJS_P2P_INJECT", "build")
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    assert c._p2p((0, 1), object(), _X()) is None
    assert c._p2p_groups[(0, 1)] is False
    assert c.p2p_fallbacks == [{"group": [0, 1], "when": "build", "reason": "injected build failure (LJS_P2P_INJECT=build)"}]
    det = c.comm_detail()
    assert det["p2p_fallbacks"][0]["when"] == "build" and det["p2p"]["groups_built"] == 0


def test_runtime_timeout_moves_job_to_rccl(monkeypatch):
    c = _comm(monkeypatch, _Dist())
    grp = _Grp(timed_out=True)
    c._p2p_groups[(0, 1)] = grp
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    monkeypatch.setattr(torch, "tensor", lambda data, dtype=None, device=None, _t=torch.tensor: _t(data, dtype=dtype))
    reason = c.p2p_health()
    assert reason and "timed out" in reason and grp.closed
    assert c._p2p_groups[(0, 1)] is False and c._p2p_off == reason
    assert c.p2p_fallbacks[0]["when"] == "runtime" and c.p2p_fallbacks[0]["group"] == [0, 1]
    # every later collective takes the bulk path, even for a group never built before
    assert c._p2p((0, 1), object(), _X()) is None and c._p2p((1, 0, 2), object(), _X()) is None
    assert c.comm_detail()["p2p"]["disabled"] == reason


def test_peer_timeout_seen_by_healthy_rank(monkeypatch):
    """This rank's groups are fine but a peer's barrier timed out: the world MAX makes every rank
    fall back together (members must agree on the path)."""
    c = _comm(monkeypatch, _Dist(peer_failed=True))
    c._p2p_groups[(0, 1)] = _Grp()
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    monkeypatch.setattr(torch, "tensor", lambda data, dtype=None, device=None, _t=torch.tensor: _t(data, dtype=dtype))
    assert c.p2p_health() == "a peer rank's p2p barrier timed out"
    assert c._p2p_off and c.p2p_fallbacks[0]["when"] == "runtime"


def test_injected_runtime_timeout(monkeypatch):
    c = _comm(monkeypatch, _Dist())
    monkeypatch.setenv("LJS_P2P_INJECT", "runtime")
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    monkeypatch.setattr(torch, "tensor", lambda data, dtype=None, device=None, _t=torch.tensor: _t(data, dtype=dtype))
    assert "injected" in c.p2p_health()
    assert c.p2p_health() is None or c._p2p_off   # once off it stays off


def test_route_log_paths(monkeypatch):
    c = _comm(monkeypatch, _Dist())
    grp = _Grp()
    c._note_route("all_reduce", (0, 1), _X(), c._p2p_path(grp, 1024, "all_reduce"))
    c._note_route("all_reduce", (0, 1), _X(), c._p2p_path(grp, 1024, "all_reduce"))
    c._note_route("all_gather", (0, 1), _X(), c._bulk_path(None))
    det = c.comm_detail()
    paths = {(r["kind"], r["path"]): r["calls"] for r in det["routes"]}
    assert paths == {("all_reduce", "p2p-oneshot"): 2, ("all_gather", "torch-nccl"): 1}
