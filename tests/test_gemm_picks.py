"""Host-side GEMM dispatch decisions (ops/hip.py cost models), pinned on the CPU."""
import pytest

from learning_jax_sharding_amd.ops import hip


@pytest.fixture
def chip(monkeypatch):
    monkeypatch.setattr(hip, "_cus", lambda: 256)
    monkeypatch.setattr(hip, "_PAIR_PICKS", {})
    monkeypatch.setattr(hip, "_DW_PAIR", "")


def test_dw_pair_one_round_equal_splits(chip):
    # the step's dW_o (20 tiles of [512 x 640]) and dW_qkv (60 tiles of [640 x 1536])
    for T, want_tile, slots in ((2048, 12884, 256), (16384, 1282, 512)):
        tile, s0, s1 = hip.pick_dw_pair(512, 640, 640, 1536, T)
        assert tile == want_tile
        assert 20 * s0 + 60 * s1 <= slots           # one round of resident blocks
        assert hip.slab_count(T // 64, s0) == s0 and hip.slab_count(T // 64, s1) == s1
    assert hip.pick_dw_pair(512, 640, 640, 1536, 16384)[1:] == (6, 6)
    assert hip.pick_dw_pair(512, 640, 640, 1536, 2048)[1:] == (3, 3)


def test_dw_pair_none_when_no_round_fits(chip):
    assert hip.pick_dw_pair(2560, 2560, 2560, 1280, 16384) is None


def test_dw_pair_forced(chip, monkeypatch):
    monkeypatch.setattr(hip, "_DW_PAIR", "11,4")
    assert hip.pick_dw_pair(512, 640, 640, 1536, 2048) == (12884, 11, 4)
    monkeypatch.setattr(hip, "_DW_PAIR", "6,6,1282")
    monkeypatch.setattr(hip, "_PAIR_PICKS", {})
    assert hip.pick_dw_pair(512, 640, 640, 1536, 2048) == (1282, 6, 6)


def test_dw_pair_ff_block_stays_separate(chip):
    # two 100-tile GEMMs (the FF block's [2560 x 640] / [640 x 2560]) would need 2-3 splits for one
    # round: the separate launches' estimate is lower
    assert hip.pick_dw_pair(2560, 640, 640, 2560, 16384) is None


def test_dw_single_picks_unchanged(chip):
    # the separate launches (a lone held GEMM, or grouping off)
    assert hip.pick_dw_slabs(640, 1536, 16384) == (1282, 8, True)
    assert hip.pick_dw_slabs(512, 640, 16384) == (1282, 16, True)   # (single-launch slab weight)
    assert hip.pick_dw_slabs(640, 1536, 2048) == (12884, 4, True)


class _FakeHip:
    """Records the grouped-launch calls of ops/linear._hold_dw (no kernels)."""

    def __init__(self, real):
        self.real, self.calls = real, []

    def __getattr__(self, name):
        return getattr(self.real, name)

    def gemm_group_begin(self):
        self.calls.append("begin")

    def gemm_group_end(self, ref):
        self.calls.append("end")


def test_held_weight_gradient_jobs_pair_and_flush(chip, monkeypatch):
    """ops/linear._hold_dw: the first slab GEMM is held, the next one launches both as a pair with
    the jointly picked split counts (inside one group), a lone held job launches alone at flush."""
    import torch
    from learning_jax_sharding_amd.ops import linear
    fake = _FakeHip(hip)
    monkeypatch.setattr(linear, "hip", fake)
    monkeypatch.setattr(linear, "_HELD", {})
    ran = []

    def job(name, K, N, T=16384):
        return linear._DwJob(K, N, T, -(-K // 128) * -(-N // 128),
                             lambda tile, S, n=name: ran.append((n, tile, S)))
    ref = torch.empty(1)
    linear._hold_dw(job("o", 512, 640), ref)
    assert ran == [] and fake.calls == []
    linear._hold_dw(job("qkv", 640, 1536), ref)
    assert fake.calls == ["begin", "end"]
    assert ran == [("o", 1282, 6), ("qkv", 1282, 6)]
    # a pair the pick declines (the FF block's): both alone with their single picks
    ran.clear()
    linear._hold_dw(job("ff_out", 2560, 640), ref)
    linear._hold_dw(job("ff_in", 640, 2560), ref)
    assert [r[0] for r in ran] == ["ff_out", "ff_in"] and fake.calls == ["begin", "end"]
    # a lone held job: launched alone when flushed
    ran.clear()
    linear._hold_dw(job("o2", 512, 640), ref)
    assert ran == []
    linear.flush_held_dw()
    assert ran == [("o2",) + tuple(hip.pick_dw_slabs(512, 640, 16384)[:2])]
    assert linear._HELD == {}
