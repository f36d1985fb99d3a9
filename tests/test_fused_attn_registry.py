"""CPU tests of the fused Q/K/V + attention plumbing (ops/hip.py register / take, ops/linear.py
gate): the attention op takes the fused forward's (o, lse) only for exactly the q / k / v column
views of the registered projection output, with the same scale, non-causal; anything else falls
back to its own kernel."""
import pytest
import torch

from learning_jax_sharding_amd.ops import hip as H
from learning_jax_sharding_amd.ops import linear as L


def _setup(B=2, Hh=4):
    T, N = B * 256, 64 * Hh
    out = torch.zeros(T, 3 * N, dtype=torch.bfloat16)
    o = torch.randn(T, N).bfloat16()
    lse = torch.randn(B, Hh, 256)
    q, k, v = (out.view(B, 256, 3, Hh, 64)[:, :, i] for i in range(3))
    return out, o, lse, q, k, v


def test_take_matches_exact_views():
    out, o, lse, q, k, v = _setup()
    H.register_fused_attention(out, o, lse, 4, 0.125)
    before = H.FUSED_ATTN_STATS["taken"]
    got = H._take_fused_attention(q, k, v, 0.125, False, 0)
    assert got is not None and H.FUSED_ATTN_STATS["taken"] == before + 1
    assert got[0].shape == (2, 256, 4, 64) and got[0].data_ptr() == o.data_ptr() and got[1] is lse
    # consumed: a second attention over the same views runs its own kernel
    assert H._take_fused_attention(q, k, v, 0.125, False, 0) is None


def test_take_refuses_mismatches():
    out, o, lse, q, k, v = _setup()
    for args in [(q, k, v, 0.25, False, 0),            # other scale
                 (q, k, v, 0.125, True, 0),            # causal
                 (q, k, v, 0.125, False, 64),          # offset queries
                 (q, v, k, 0.125, False, 0),           # k / v swapped
                 (q.contiguous(), k, v, 0.125, False, 0)]:   # a copy of q
        H.register_fused_attention(out, o, lse, 4, 0.125)
        assert H._take_fused_attention(*args) is None
    # written after registration (version bump): stale, not taken
    H.register_fused_attention(out, o, lse, 4, 0.125)
    out.add_(0)
    assert H._take_fused_attention(q, k, v, 0.125, False, 0) is None
    H._FUSED_ATTN.clear()


def test_gate_needs_announcement_and_shapes():
    x = torch.zeros(2, 256, 640)
    xb = torch.zeros(512, 640, dtype=torch.bfloat16)
    wt = torch.zeros(3, 512, 640, dtype=torch.bfloat16)
    args = (x, xb, wt, 3, 512, 640, None, False, None, torch.bfloat16, torch.bfloat16, False, (0, 1, 2), False)
    assert L._fuse_attention_ok(*args) is None                  # not announced
    with L.attention_next(8, 64, 0.125):
        assert L._fuse_attention_ok(*args) is None              # CPU tensors
        assert L._ATTN_NEXT[0] == (8, 64, 0.125)
    assert L._ATTN_NEXT[0] is None
    old = L._QKV_ATTN
    try:
        L._QKV_ATTN = False
        with L.attention_next(8, 64, 0.125):
            assert L._ATTN_NEXT[0] is None                      # LJS_QKV_ATTN=0
    finally:
        L._QKV_ATTN = old


def test_capture_end_drops_untaken_forward():
    from learning_jax_sharding_amd.spmd import graphs
    out, o, lse, q, k, v = _setup()
    H.register_fused_attention(out, o, lse, 4, 0.125)
    assert H.clear_fused_attention in graphs.AFTER_CAPTURE
    for f in graphs.AFTER_CAPTURE:
        if f is H.clear_fused_attention:
            f()
    assert H._take_fused_attention(q, k, v, 0.125, False, 0) is None


def test_attention_head_dim_dispatch(monkeypatch):
    """GPU attention entry points take the HIP kernels for head_dim 64 with a contiguous last dim
    and the torch formulation (warned once per head-dim pair) for anything else."""
    import warnings

    import torch

    from learning_jax_sharding_amd.ops import kernels as K
    monkeypatch.setattr(K, "use_hip", lambda t: True)
    monkeypatch.setattr(K, "_WARNED_DH", set())
    q64 = torch.zeros(1, 4, 2, 64)
    assert K._hip_attn(q64, q64, q64)
    strided = torch.zeros(1, 4, 2, 128)[..., ::2]
    with pytest.warns(UserWarning, match="head_dim 64"):
        assert not K._hip_attn(strided, strided, strided)
    q32 = torch.zeros(1, 4, 2, 32)
    with pytest.warns(UserWarning, match="head_dim 32"):
        assert not K._hip_attn(q32, q32, q32)
    with warnings.catch_warnings():
        warnings.simplefilter("error")     # once per head-dim pair
        assert not K._hip_attn(q32, q32, q32)
