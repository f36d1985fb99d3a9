"""HIP kernel numerics vs plain PyTorch fp32 references (run on a real MI355X: -m gpu)."""
import os
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

dev = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def hip():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from learning_jax_sharding_amd.ops import hip as H
    H.lib()
    return H


def _rand(*shape, dtype=torch.bfloat16, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(*shape, generator=g).to(dtype).to(dev)


def _stored(mat, kc_rowmajor: bool):
    """Return (storage tensor, ld) for a logical [R][K] matrix in KC or MN-contiguous layout."""
    if kc_rowmajor:
        return mat.contiguous(), mat.shape[1]
    return mat.t().contiguous(), mat.shape[0]


@pytest.mark.parametrize("a_kc,b_kc", [(1, 1), (0, 0), (1, 0), (0, 1)])
@pytest.mark.parametrize("out_f32", [0, 1])
@pytest.mark.parametrize("tile", [64, 128, 2561, 2562, 1284, 1282, 12883, 12884, 1602, 643, 644, 2563, 12856])
@pytest.mark.parametrize("M,N,K", [(256, 192, 320), (136, 72, 40), (512, 1536, 640), (304, 136, 128), (384, 640, 512)])
def test_gemm_layouts(hip, a_kc, b_kc, out_f32, tile, M, N, K):
    A = _rand(M, K, seed=1)
    B = _rand(K, N, seed=2)
    ref = A.float() @ B.float()
    As, lda = _stored(A, a_kc)               # KC: [M][K]; MN: [K][M]
    Bs, ldb = _stored(B.t(), b_kc)           # KC: [N][K]; MN: [K][N]
    C = torch.full((M, N), float("nan"), dtype=torch.float32 if out_f32 else torch.bfloat16, device=dev)
    hip.gemm(As, Bs, C, M, N, K, lda, ldb, N, bool(a_kc), bool(b_kc), tile=tile)
    torch.cuda.synchronize()
    tol = 2e-2 if not out_f32 else 1e-3
    torch.testing.assert_close(C.float(), ref, rtol=tol, atol=tol * math.sqrt(K))


@pytest.mark.parametrize("tile", [1284, 1282, 2561, 12883, 12884])
def test_gemm_dma_splitk_batched_broadcast(hip, tile):
    """LDS-DMA kernels: weight-grad layout (both operands m/n-contiguous) with split-K atomics
    into a zeroed f32 C, batched column blocks, and a broadcast (ld = 0) k-contiguous row."""
    T, M, N, nb = 2048, 320, 128, 3
    X = _rand(T, M, seed=7)
    dY = _rand(T, nb * N, seed=8)
    dW = torch.full((nb, M, N), float("nan"), dtype=torch.float32, device=dev)
    hip.gemm(X, dY, dW, M, N, T, M, nb * N, N, False, False, batch=nb, sA=0, sB=N, sC=M * N, splitk=4,
             tile=tile, zero_c=True)
    for i in range(nb):
        torch.testing.assert_close(dW[i], X.float().t() @ dY[:, i * N:(i + 1) * N].float(), rtol=1e-3, atol=5e-2)
    row = _rand(1, 256, seed=9)
    W = _rand(320, 256, seed=10)
    out = torch.empty((500, 320), dtype=torch.bfloat16, device=dev)
    hip.gemm(row, W, out, 500, 320, 256, 0, 256, 320, True, True, tile=tile)
    torch.testing.assert_close(out.float(), (row.float() @ W.float().t()).expand(500, 320), rtol=2e-2, atol=5e-2)


@pytest.mark.parametrize("M", [1024, 1000])
def test_gemm_tile2562_folded_batch(hip, M):
    """256x192 tile: a weight-major batch of 3 side by side in C (the fused Q/K/V projection) is
    folded into one GEMM over 3N columns; ragged rows; bit-identical to the 256x128 kernel (same
    k order per output element)."""
    N, K, nb = 512, 640, 3
    x = _rand(M, K, seed=21)
    w = _rand(nb, N, K, seed=22)
    out = torch.full((M, nb * N), float("nan"), dtype=torch.bfloat16, device=dev)
    hip.gemm(x, w, out, M, N, K, K, K, nb * N, True, True, batch=nb, sA=0, sB=N * K, sC=N, tile=2562)
    ref = torch.full_like(out, float("nan"))
    hip.gemm(x, w, ref, M, N, K, K, K, nb * N, True, True, batch=nb, sA=0, sB=N * K, sC=N, tile=2561)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    f = torch.einsum("mk,bnk->mbn", x.float(), w.float()).reshape(M, nb * N)
    torch.testing.assert_close(out.float(), f, rtol=2e-2, atol=2e-2 * math.sqrt(K))


def test_gemm_identity_asymmetric(hip):
    """A = I with an asymmetric B catches a transposed C write."""
    n = 64
    A = torch.eye(n, dtype=torch.bfloat16, device=dev)
    B = (torch.arange(n * n, device=dev).reshape(n, n) % 97).to(torch.bfloat16)
    C = torch.empty((n, n), dtype=torch.float32, device=dev)
    hip.gemm(A, B.t().contiguous(), C, n, n, n, n, n, n, True, True)
    torch.testing.assert_close(C, B.float())


def test_gemm_bias_relu_batched_splitk(hip):
    M, N, K, nb = 128, 256, 512, 3
    A = _rand(M, K, seed=3)
    Bt = _rand(nb, N, K, seed=4)
    bias = _rand(N, dtype=torch.float32, seed=5)
    out = torch.empty((M, nb * N), dtype=torch.bfloat16, device=dev)
    hip.gemm(A, Bt, out, M, N, K, K, K, nb * N, True, True, batch=nb, sA=0, sB=N * K, sC=N, bias=bias, relu=True)
    ref = torch.relu(torch.einsum("mk,bnk->bmn", A.float(), Bt.float()) + bias)
    for i in range(nb):
        torch.testing.assert_close(out[:, i * N:(i + 1) * N].float(), ref[i], rtol=2e-2, atol=5e-2)
    # split-K accumulation into f32
    C = torch.zeros((M, N), dtype=torch.float32, device=dev)
    hip.gemm(A, Bt[0], C, M, N, K, K, K, N, True, True, splitk=4)
    torch.testing.assert_close(C, A.float() @ Bt[0].float().t(), rtol=1e-3, atol=1e-2)


def test_gemm_f32_strided(hip):
    A = torch.randn(3, 20, 36, device=dev)
    B = torch.randn(3, 36, 12, device=dev)
    C = torch.empty(3, 20, 12, device=dev)
    hip._gemm_f32(A, B, C, 20, 12, 36, 36, 1, 12, 1, 12, 20 * 36, 36 * 12, 20 * 12, 3)
    torch.testing.assert_close(C, A @ B, rtol=1e-5, atol=1e-4)
    # transposed operand through strides
    At = A.transpose(1, 2).contiguous()
    hip._gemm_f32(At, B, C, 20, 12, 36, 1, 20, 12, 1, 12, 20 * 36, 36 * 12, 20 * 12, 3)
    torch.testing.assert_close(C, A @ B, rtol=1e-5, atol=1e-4)


def test_bmm_nt_autograd(hip):
    for dt in (torch.float32, torch.bfloat16):
        A = torch.randn(2, 24, 40, device=dev, dtype=dt, requires_grad=True)
        Bt = torch.randn(2, 16, 40, device=dev, dtype=dt, requires_grad=True)
        C = hip.bmm_nt(A, Bt, torch.float32)
        g = torch.randn_like(C)
        (C * g).sum().backward()
        A2 = A.detach().float().requires_grad_()
        B2 = Bt.detach().float().requires_grad_()
        C2 = A2 @ B2.transpose(1, 2)
        (C2 * g).sum().backward()
        tol = 1e-4 if dt == torch.float32 else 3e-2
        torch.testing.assert_close(C, C2, rtol=tol, atol=tol * 10)
        torch.testing.assert_close(A.grad.float(), A2.grad, rtol=tol, atol=tol * 10)
        torch.testing.assert_close(Bt.grad.float(), B2.grad, rtol=tol, atol=tol * 10)


def _attn_ref(q, k, v, scale, causal=False, q_offset=0):
    from learning_jax_sharding_amd.ops.kernels import attention_reference
    return attention_reference(q, k, v, scale, causal, q_offset)


@pytest.fixture(params=["fused", "split"])
def attn_bwd_impl(request, hip):
    hip.set_attention_bwd_fused(request.param == "fused")
    yield request.param
    hip.set_attention_bwd_fused(None)


@pytest.fixture(params=[(1, 0), (1, 4), (1, 8)], ids=["tiled1", "res4", "res8"])
def attn_fwd_nsub(request, hip):
    """Forward kernel variant: tiled (K/V tiles through registers), or K/V-resident with 4 / 8
    waves per block (Sk <= 256; longer keys fall back to the tiled kernel)."""
    _, res = request.param
    hip.set_attention_fwd_resident(res)
    yield request.param
    hip.set_attention_fwd_resident(-1)


@pytest.mark.parametrize("B,S,H", [(2, 256, 8), (1, 200, 4), (3, 64, 2), (1, 40, 3), (1, 320, 2)])
@pytest.mark.parametrize("causal", [False, True])
def test_attention_fwd_bwd(hip, attn_bwd_impl, attn_fwd_nsub, B, S, H, causal):
    D = 64
    # q/k/v as column slices of one fused QKV buffer, exactly as the model produces them
    qkv = _rand(B, S, 3 * H * D, seed=7).reshape(B, S, 3, H, D)
    q, k, v = (qkv[:, :, i] for i in range(3))
    scale = D ** -0.5
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    ref = _attn_ref(qr, kr, vr, scale, causal).float()
    out = hip.attention(q, k, v, scale, causal)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    # backward vs autograd of the f32 reference
    q1, k1, v1 = (t.detach().clone().requires_grad_() for t in (q, k, v))
    out1 = hip.attention(q1, k1, v1, scale, causal)
    g = _rand(*out1.shape, seed=9)
    (out1.float() * g.float()).sum().backward()
    s = torch.einsum("btnh,bfnh->bnft", kr, qr) * scale
    if causal:
        s = s.masked_fill(torch.arange(S, device=dev)[None, :] > torch.arange(S, device=dev)[:, None], -float("inf"))
    o = torch.einsum("bnft,btnh->bfnh", torch.softmax(s, -1), vr)
    (o * g.float()).sum().backward()
    for a, b_, name in ((q1.grad, qr.grad, "dq"), (k1.grad, kr.grad, "dk"), (v1.grad, vr.grad, "dv")):
        err = (a.float() - b_).abs().max().item()
        assert err <= 3e-2 * max(1.0, b_.abs().max().item()), (name, err)


@pytest.mark.parametrize("B,S,H,causal", [(16, 256, 8, False), (2, 256, 8, False), (16, 200, 8, True),
                                           (3, 100, 3, False), (1, 320, 2, True)])
def test_attention_vst_bit_exact(hip, B, S, H, causal):
    """Row tiles stored through the LDS image (16-byte whole-row stores: resident forward, fused
    and 128-key split backward) == the per-lane 8-byte stores, bit for bit, with ragged Sq."""
    D = 64
    qkv = _rand(B, S, 3 * H * D, seed=11).reshape(B, S, 3, H, D)
    g = _rand(B, S, H, D, seed=12)
    res = {}
    for vst in (True, False):
        hip.set_attention_vst(vst)
        q, k, v = (qkv[:, :, i].detach().clone().requires_grad_() for i in range(3))
        o = hip.attention(q, k, v, D ** -0.5, causal)
        (o.float() * g.float()).sum().backward()
        res[vst] = (o.detach(), q.grad, k.grad, v.grad)
    hip.set_attention_vst(None)
    for a, b_, name in zip(res[True], res[False], ("o", "dq", "dk", "dv")):
        assert torch.equal(a, b_), name


@pytest.mark.parametrize("Sq,Sk,causal,q_offset", [(192, 128, False, 0), (130, 256, True, 64), (64, 100, True, 0)])
def test_attention_bwd_block_fused_matches_split(hip, attn_fwd_nsub, Sq, Sk, causal, q_offset):
    """Block backward (ring attention's kernel: external O / lse, Sq != Sk, causal offset):
    the fused single-pass kernel == the split dQ + dK/dV kernels."""
    B, H, D = 2, 3, 64
    q, do = _rand(B, Sq, H, D, seed=1), _rand(B, Sq, H, D, seed=2)
    k, v = _rand(B, Sk, H, D, seed=3), _rand(B, Sk, H, D, seed=4)
    o, lse = hip.attn_fwd_lse(q, k, v, D ** -0.5, causal, q_offset)
    outs = {}
    for fused in (True, False):
        hip.set_attention_bwd_fused(fused)
        outs[fused] = hip.attn_bwd_block(q, k, v, o, do, lse, D ** -0.5, causal, q_offset)
    hip.set_attention_bwd_fused(None)
    for a, b_ in zip(outs[True], outs[False]):
        torch.testing.assert_close(a.float(), b_.float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("B,Sq,Sk,H,causal,q_offset", [(4, 128, 256, 8, False, 0), (2, 256, 256, 4, False, 0),
                                                     (2, 192, 128, 3, False, 0), (2, 130, 256, 3, True, 64)])
def test_attention_bwd_fused_kv_dma_bit_exact(hip, B, Sq, Sk, H, causal, q_offset):
    """Fused backward with K / V staged by LDS-DMA (both sweep instances: the one-sweep common
    case at Sk == 256 and the general one) == the register-staged copy, bit for bit."""
    D = 64
    q, do = _rand(B, Sq, H, D, seed=1), _rand(B, Sq, H, D, seed=2)
    k, v = _rand(B, Sk, H, D, seed=3), _rand(B, Sk, H, D, seed=4)
    o, lse = hip.attn_fwd_lse(q, k, v, D ** -0.5, causal, q_offset)
    hip.set_attention_bwd_fused(True)
    outs = {}
    try:
        for kv in (True, False):
            hip.set_attention_bwd_kv_dma(kv)
            outs[kv] = hip.attn_bwd_block(q, k, v, o, do, lse, D ** -0.5, causal, q_offset)
    finally:
        hip.set_attention_bwd_kv_dma(None)
        hip.set_attention_bwd_fused(None)
    for a, b_, name in zip(outs[True], outs[False], ("dq", "dk", "dv")):
        assert torch.equal(a, b_), name


@pytest.mark.parametrize("B,Sq,Sk,H,causal,q_offset", [(8, 256, 256, 8, False, 0), (2, 192, 128, 3, False, 0),
                                                     (2, 130, 256, 3, True, 64), (1, 64, 100, 2, True, 0)])
def test_attention_bwd_pair_matches_two_launches(hip, B, Sq, Sk, H, causal, q_offset):
    """The split backward as one launch (dQ and dK/dV blocks side by side, the dK/dV blocks
    forming delta = rowsum(dO o O) themselves) == the dQ kernel then the dK/dV kernel: dQ
    bit-exact (same code), dK/dV up to delta's f32 summation order."""
    D = 64
    q, do = _rand(B, Sq, H, D, seed=1), _rand(B, Sq, H, D, seed=2)
    k, v = _rand(B, Sk, H, D, seed=3), _rand(B, Sk, H, D, seed=4)
    o, lse = hip.attn_fwd_lse(q, k, v, D ** -0.5, causal, q_offset)
    hip.set_attention_bwd_fused(False)
    hip.set_attention_dkv32(False)  # the 64-row blocks (128-row ones: test_attention_bwd_dkv32_*)
    outs = {}
    try:
        for pair in (True, False):
            hip.set_attention_bwd_pair(pair)
            outs[pair] = hip.attn_bwd_block(q, k, v, o, do, lse, D ** -0.5, causal, q_offset)
    finally:
        hip.set_attention_bwd_pair(None)
        hip.set_attention_dkv32(None)
        hip.set_attention_bwd_fused(None)
    assert torch.equal(outs[True][0], outs[False][0])
    for a, b_ in zip(outs[True][1:], outs[False][1:]):
        torch.testing.assert_close(a.float(), b_.float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("B,Sq,Sk,H,causal,q_offset", [(1, 1024, 1024, 2, False, 0), (2, 320, 320, 3, True, 0),
                                                     (1, 200, 700, 2, True, 500), (2, 192, 130, 2, False, 0),
                                                     (1, 64, 100, 2, True, 0)])
@pytest.mark.parametrize("dq32", [True, False])
def test_attention_bwd_dkv32_matches_dkv16(hip, B, Sq, Sk, H, causal, q_offset, dq32):
    """Split backward with 128-key dK/dV blocks (32 keys per wave, LDS-DMA query tiles) and 64- or
    128-query dQ blocks (32 queries per wave) == the 64-key / 64-query blocks: dQ bit-exact (same
    per-query sums in the same order), dK/dV up to delta's f32 summation order; and against
    autograd of the f32 reference."""
    D = 64
    scale = D ** -0.5
    q, do = _rand(B, Sq, H, D, seed=11), _rand(B, Sq, H, D, seed=12)
    k, v = _rand(B, Sk, H, D, seed=13), _rand(B, Sk, H, D, seed=14)
    o, lse = hip.attn_fwd_lse(q, k, v, scale, causal, q_offset)
    hip.set_attention_bwd_fused(False)
    hip.set_attention_dq32(dq32)
    outs = {}
    try:
        for d32 in (True, False):
            hip.set_attention_dkv32(d32)
            outs[d32] = hip.attn_bwd_block(q, k, v, o, do, lse, scale, causal, q_offset)
    finally:
        hip.set_attention_dkv32(None)
        hip.set_attention_dq32(None)
        hip.set_attention_bwd_fused(None)
    assert torch.equal(outs[True][0], outs[False][0])
    for a, b_ in zip(outs[True][1:], outs[False][1:]):
        torch.testing.assert_close(a.float(), b_.float(), rtol=1e-2, atol=1e-2)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    (_attn_ref(qr, kr, vr, scale, causal, q_offset).float() * do.float()).sum().backward()
    for a, b_, name in zip(outs[True], (qr.grad, kr.grad, vr.grad), ("dq", "dk", "dv")):
        err = (a.float() - b_).abs().max().item()
        assert err <= 3e-2 * max(1.0, b_.abs().max().item()), (name, err)


def test_attention_online_softmax_rescale(hip):
    """Force a running-max jump at a late key tile (exercises the rescale branch)."""
    B, S, H, D = 1, 256, 1, 64
    q = torch.zeros(B, S, H, D, device=dev, dtype=torch.bfloat16)
    k = torch.zeros_like(q)
    v = _rand(B, S, H, D, seed=3)
    q[:, :, :, 0] = 1.0
    k[:, 200, :, 0] = 40.0  # one very large score in the 4th key tile
    out = hip.attention(q, k, v, D ** -0.5)
    ref = _attn_ref(q, k, v, D ** -0.5)
    torch.testing.assert_close(out.float(), ref.float(), rtol=2e-2, atol=2e-2)


def test_elementwise(hip):
    x = torch.randn(1000003, device=dev)
    torch.testing.assert_close(hip.cast(x, torch.bfloat16), x.bfloat16())
    xb = x.bfloat16()
    torch.testing.assert_close(hip.cast(xb, torch.float32), xb.float())
    torch.testing.assert_close(hip.sum_all(x, torch.float32), x.sum(), rtol=1e-4, atol=1e-2)
    m = torch.randn(333, 77, device=dev)
    torch.testing.assert_close(hip.colsum(m), m.sum(0), rtol=1e-5, atol=1e-4)
    s = torch.randn(17, 300, device=dev)
    torch.testing.assert_close(hip.softmax_lastdim(s), torch.softmax(s, -1), rtol=1e-5, atol=1e-6)
    w = torch.randn(640, 512, device=dev)
    torch.testing.assert_close(hip.cast_transpose_bf16(w), w.t().bfloat16(), rtol=0, atol=0)
    for R, C in ((320, 512), (37, 70), (1, 33), (65, 1)):   # ragged tiles, scalar tails
        w = torch.randn(R, C, device=dev)
        torch.testing.assert_close(hip.cast_transpose_bf16(w), w.t().bfloat16(), rtol=0, atol=0)
    w = torch.randn(96, 130, device=dev)[:, 1:129]          # row stride 130, 4-byte-aligned base
    torch.testing.assert_close(hip.cast_transpose_bf16(w), w.t().bfloat16(), rtol=0, atol=0)


def test_adam_kernel(hip):
    p = torch.randn(4099, device=dev)
    g = torch.randn(4099, device=dev)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    tp = p.clone().requires_grad_()
    opt = torch.optim.Adam([tp], lr=1e-3)
    step = torch.zeros((), dtype=torch.int32, device=dev)
    for i in range(3):
        step += 1
        p, m, v = hip.adam(p, g, m, v, step, 1e-3, 0.9, 0.999, 1e-8, 0.0, inplace=True)
        tp.grad = g.clone()
        opt.step()
    torch.testing.assert_close(p, tp.detach(), rtol=1e-5, atol=1e-6)


def test_rng_matches_host(hip):
    import learning_jax_sharding_amd.random as R
    k = R.PRNGKey(3)
    for dist, lo, hi in (("normal", 0, 1), ("uniform", -2, 3), ("truncated_normal", -2, 2)):
        shape = (6, 10)
        region = ((2, 5), (4, 10))
        gpu = hip.rng_fill(shape, region, k.k0, k.k1, dist, lo, hi, torch.float32, dev).cpu().numpy()
        idx = (np.arange(2, 5)[:, None] * 10 + np.arange(4, 10)[None, :]).astype(np.uint64)
        host = R._dist_np(idx.reshape(-1), k, dist, lo, hi).reshape(idx.shape)
        np.testing.assert_allclose(gpu, host, rtol=1e-5, atol=1e-5)


def test_linear_autograd(hip):
    x = _rand(256, 640, dtype=torch.float32, seed=11).requires_grad_()
    ws = [(_rand(640, 512, dtype=torch.float32, seed=20 + i) * 0.05).requires_grad_() for i in range(3)]
    ys = hip.linear(x, ws, None, torch.bfloat16, False, torch.bfloat16)
    gs = [_rand(256, 512, seed=30 + i) for i in range(3)]
    sum((y.float() * g.float()).sum() for y, g in zip(ys, gs)).backward()
    xr = x.detach().clone().requires_grad_()
    wr = [w.detach().clone().requires_grad_() for w in ws]
    yr = [xr.bfloat16().float() @ w.bfloat16().float() for w in wr]
    sum((y * g.float()).sum() for y, g in zip(yr, gs)).backward()
    for y, r in zip(ys, yr):
        torch.testing.assert_close(y.float(), r, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(x.grad, xr.grad, rtol=3e-2, atol=3e-2)
    for w, r in zip(ws, wr):
        torch.testing.assert_close(w.grad, r.grad, rtol=3e-2, atol=3e-1)
    # bias + relu path
    b = _rand(512, dtype=torch.float32, seed=40).requires_grad_()
    (y,) = hip.linear(x, [ws[0]], b, torch.bfloat16, True, torch.bfloat16)
    y.float().sum().backward()
    yr = torch.relu(xr.bfloat16().float() @ wr[0].bfloat16().float() + b.detach().bfloat16().float())
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(b.grad, (yr > 0).float().sum(0), rtol=1e-2, atol=2.0)


def test_adam_multi_and_shadows(hip):
    from learning_jax_sharding_amd.ops import shadow
    ws = [torch.randn(640, 512, device=dev), torch.randn(512, 640, device=dev), torch.randn(640, device=dev)]
    gs = [torch.randn_like(w) for w in ws]
    ms = [torch.zeros_like(w) for w in ws]
    vs = [torch.zeros_like(w) for w in ws]
    refs = [w.clone().requires_grad_() for w in ws]
    opt = torch.optim.Adam(refs, lr=1e-3)
    shadow.get(ws[0], "T")
    shadow.get(ws[1], "N")
    step = torch.zeros((), dtype=torch.int32, device=dev)
    for _ in range(2):
        step += 1
        hip.adam_multi(list(zip(ws, gs, ms, vs)), step, 1e-3, 0.9, 0.999, 1e-8, 0.0)
        for r, g in zip(refs, gs):
            r.grad = g.clone()
        opt.step()
    for w, r in zip(ws, refs):
        torch.testing.assert_close(w, r.detach(), rtol=1e-5, atol=1e-6)
    # shadows were refreshed by the kernel (no re-cast needed) and equal the new weights
    e0 = shadow.entry(ws[0], create=False)
    assert e0.versions["T"] == ws[0]._version
    torch.testing.assert_close(e0.bufs["T"], ws[0].t().bfloat16())
    torch.testing.assert_close(shadow.entry(ws[1], create=False).bufs["N"], ws[1].bfloat16())


@pytest.mark.parametrize("S", [3, 7, 11, 24])
def test_adam_multi_slab_grads_bit_exact(hip, S):
    """Adam reading split-K slabs directly (the kernel's slab sum, double-buffered in <= 32-row
    tiles of the default 32-row launch) equals slab_reduce + Adam on the combined gradient, bit for bit."""
    shapes = [(640, 512), (512, 640)]
    ws = [torch.randn(*sh, device=dev) for sh in shapes]
    slabs = [torch.randn(S, *sh, device=dev) for sh in shapes]
    ms = [torch.rand(*sh, device=dev) * 1e-2 for sh in shapes]
    vs = [torch.rand(*sh, device=dev) * 1e-3 for sh in shapes]
    w2, m2, v2 = [w.clone() for w in ws], [m.clone() for m in ms], [v.clone() for v in vs]
    step = torch.full((), 3, dtype=torch.int32, device=dev)
    gsl = [hip.SlabGrad(sl, S, 0, sh[1], sh[0] * sh[1], sh) for sl, sh in zip(slabs, shapes)]
    hip.adam_multi(list(zip(ws, gsl, ms, vs)), step, 1e-3, 0.9, 0.999, 1e-8, 0.0)
    gc = []
    for sl, sh in zip(slabs, shapes):
        g = torch.empty(*sh, device=dev)
        hip.slab_reduce(sl, g, sh[1], sh[0] * sh[1])
        gc.append(g)
    hip.adam_multi(list(zip(w2, gc, m2, v2)), step, 1e-3, 0.9, 0.999, 1e-8, 0.0)
    torch.cuda.synchronize()
    for a, b in zip(ws + ms + vs, w2 + m2 + v2):
        assert torch.equal(a, b)


@pytest.mark.parametrize("S", [8, 12, 16])
def test_adam_multi_short_tiles_with_shadows(hip, S):
    """Tensors with >= 2x the slabs of the launch's lightest slab gradient run in 32-row tiles
    (>= 4x: 16-row) chosen per tensor in the same launch as 64-row ones (here 4 slabs vs S): p/m/v
    and both bf16 shadows equal slab_reduce + Adam on the combined gradient (64-row tiles), bit
    for bit."""
    from learning_jax_sharding_amd.ops import shadow
    shapes = [(640, 512), (512, 640), (200, 128)]
    Ss = [4, S, S]
    ws = [torch.randn(*sh, device=dev) for sh in shapes]
    slabs = [torch.randn(k, *sh, device=dev) for k, sh in zip(Ss, shapes)]
    ms = [torch.rand(*sh, device=dev) * 1e-2 for sh in shapes]
    vs = [torch.rand(*sh, device=dev) * 1e-3 for sh in shapes]
    w2, m2, v2 = [w.clone() for w in ws], [m.clone() for m in ms], [v.clone() for v in vs]
    for w in ws + w2:
        shadow.get(w, "T")
        shadow.get(w, "N")
    step = torch.full((), 5, dtype=torch.int32, device=dev)
    gsl = [hip.SlabGrad(sl, k, 0, sh[1], sh[0] * sh[1], sh) for sl, k, sh in zip(slabs, Ss, shapes)]
    hip.adam_multi(list(zip(ws, gsl, ms, vs)), step, 1e-3, 0.9, 0.999, 1e-8, 0.01)
    gc = []
    for sl, sh in zip(slabs, shapes):
        g = torch.empty(*sh, device=dev)
        hip.slab_reduce(sl, g, sh[1], sh[0] * sh[1])
        gc.append(g)
    hip.adam_multi(list(zip(w2, gc, m2, v2)), step, 1e-3, 0.9, 0.999, 1e-8, 0.01)
    torch.cuda.synchronize()
    for a, b in zip(ws + ms + vs, w2 + m2 + v2):
        assert torch.equal(a, b)
    for a, b in zip(ws, w2):
        ea, eb = shadow.entry(a, create=False), shadow.entry(b, create=False)
        for kind in ("T", "N"):
            assert torch.equal(ea.bufs[kind].view(torch.int16), eb.bufs[kind].view(torch.int16)), kind
        assert torch.equal(ea.bufs["T"], a.t().bfloat16())


@pytest.mark.parametrize("with_bf16", [False, True])
def test_adam_multi_mx_shadows(hip, with_bf16):
    """The fused Adam rewrites a weight's MX-fp8 shadows (blocks along rows and, transposed,
    along columns) bit-exactly equal to quantizing the updated weight, and marks them fresh."""
    from learning_jax_sharding_amd.ops import fp8 as F, shadow
    ws = [torch.randn(640, 2560, device=dev) * 0.05, torch.randn(2560, 640, device=dev) * 0.03]
    gs = [torch.randn_like(w) for w in ws]
    ms = [torch.zeros_like(w) for w in ws]
    vs = [torch.zeros_like(w) for w in ws]
    for w in ws:
        assert shadow.mx_eligible(w)
        shadow.get_mx(w, "QT")
        shadow.get_mx(w, "QN")
        if with_bf16:
            shadow.get(w, "T")
    step = torch.zeros((), dtype=torch.int32, device=dev)
    for _ in range(2):
        hip.adam_multi(list(zip(ws, gs, ms, vs)), step, 1e-3, 0.9, 0.999, 1e-8, 0.0, increment_step=True)
    torch.cuda.synchronize()
    for w in ws:
        e = shadow.entry(w, create=False)
        assert e.versions["QT"] == w._version and e.versions["QN"] == w._version
        qt, st = F.quant_cols(w)
        qn, sn = F.quant_rows(w)
        assert torch.equal(e.bufs["QT"], qt) and torch.equal(e.bufs["QTs"], st)
        assert torch.equal(e.bufs["QN"], qn) and torch.equal(e.bufs["QNs"], sn)
        assert shadow.get_mx(w, "QT")[0].data_ptr() == e.bufs["QT"].data_ptr()  # no re-quantization
        if with_bf16:
            torch.testing.assert_close(e.bufs["T"], w.t().bfloat16())


@pytest.mark.parametrize("R,C", [(640, 512), (200, 132), (96, 100), (70, 66), (33, 7)])
@pytest.mark.parametrize("g_bf16", [False, True])
def test_adam_multi_vector_and_edges(hip, R, C, g_bf16):
    """Adam's 4-wide path (C % 4 == 0, aligned; ragged row/column tiles fall back per tile) and the
    scalar path agree with torch.optim.Adam, bf16 gradients included, and both bf16 shadows
    (plain and transposed) equal the updated weights."""
    from learning_jax_sharding_amd.ops import shadow
    w = torch.randn(R, C, device=dev)
    g = torch.randn(R, C, device=dev)
    if g_bf16:
        g = g.bfloat16()
    m, v = torch.zeros_like(w), torch.zeros_like(w)
    ref = w.clone().requires_grad_()
    opt = torch.optim.Adam([ref], lr=1e-3)
    shadow.get(w, "T")
    shadow.get(w, "N")
    step = torch.zeros((), dtype=torch.int32, device=dev)
    for _ in range(3):
        step += 1
        hip.adam_multi([(w, g, m, v)], step, 1e-3, 0.9, 0.999, 1e-8, 0.0)
        ref.grad = g.float().clone()
        opt.step()
    torch.testing.assert_close(w, ref.detach(), rtol=1e-5, atol=1e-6)
    e = shadow.entry(w, create=False)
    torch.testing.assert_close(e.bufs["T"], w.t().bfloat16())
    torch.testing.assert_close(e.bufs["N"], w.bfloat16())


def test_linear_broadcast_grad_and_strided(hip):
    """dY that repeats one row (cotangent of y.sum()) is read with ld=0, not materialised."""
    x = _rand(128, 256, dtype=torch.float32, seed=1)
    w = (_rand(256, 320, dtype=torch.float32, seed=2) * 0.05).requires_grad_()
    b = torch.zeros(320, device=dev, requires_grad=True)
    xr = x.clone().requires_grad_()
    (y,) = hip.linear(xr, [w], b, torch.bfloat16, False, torch.bfloat16)
    y.float().sum().backward()
    xf = x.bfloat16().float()
    torch.testing.assert_close(w.grad, xf.sum(0)[:, None].expand(256, 320), rtol=1e-2, atol=1e-1)
    torch.testing.assert_close(b.grad, torch.full((320,), 128.0, device=dev))
    torch.testing.assert_close(xr.grad, w.detach().bfloat16().float().sum(1)[None, :].expand(128, 256),
                               rtol=2e-2, atol=5e-2)


def test_linear_scalar_broadcast_grad(hip):
    """The cotangent of the bf16 sum_all is the seed scalar broadcast with all strides 0: the
    dense backward turns it into its bf16 row + bias gradient in one kernel (bcast_scalar)."""
    x = _rand(256, 256, dtype=torch.float32, seed=3)
    w = (_rand(256, 320, dtype=torch.float32, seed=4) * 0.05).requires_grad_()
    b = torch.zeros(320, device=dev, requires_grad=True)
    xr = x.clone().requires_grad_()
    (y,) = hip.linear(xr, [w], b, torch.bfloat16, False, torch.bfloat16)
    s = hip.sum_all(y, torch.bfloat16)
    seed = torch.tensor(0.5, dtype=torch.bfloat16, device=dev)
    gw, gb, gx = torch.autograd.grad(s, [w, b, xr], seed)
    xf = x.bfloat16().float()
    torch.testing.assert_close(gw, 0.5 * xf.sum(0)[:, None].expand(256, 320), rtol=1e-2, atol=1e-1)
    torch.testing.assert_close(gb, torch.full((320,), 128.0, device=dev))
    torch.testing.assert_close(gx, 0.5 * w.detach().bfloat16().float().sum(1)[None, :].expand(256, 256),
                               rtol=2e-2, atol=5e-2)


@pytest.mark.parametrize("T,N", [(16384, 640), (4096, 512), (1000, 1152)])
def test_fused_output_sum(hip, T, N):
    """A large bf16 dense output carries its per-tile sums from the GEMM epilogue; sum_all of it
    reduces those partials (== the sum of the stored bf16 values), and falls back to reading
    the array once the output was modified in place or only part of it is summed."""
    x = _rand(T, 640, dtype=torch.float32, seed=5)
    w = _rand(640, N, dtype=torch.float32, seed=6) * 0.05
    b = _rand(N, dtype=torch.float32, seed=7)
    (y,) = hip.linear(x, [w], b, torch.bfloat16, False, torch.bfloat16)
    fused = hip._psum_for(y) is not None
    ref = y.float().sum()
    got = hip.sum_all(y, torch.bfloat16)
    torch.testing.assert_close(got.float(), ref, rtol=1e-2, atol=1.0)
    got32 = hip.sum_all(y, torch.float32)
    torch.testing.assert_close(got32, ref, rtol=1e-4, atol=1e-1)
    if T * N >= (1 << 20) and T % 64 == 0:
        assert fused, "expected the DMA GEMM to produce fused partial sums"
    y.mul_(2.0)
    assert hip._psum_for(y) is None
    torch.testing.assert_close(hip.sum_all(y, torch.float32), 2 * ref, rtol=1e-4, atol=2e-1)
    half = y[: T // 2]
    torch.testing.assert_close(hip.sum_all(half, torch.float32), half.float().sum(), rtol=1e-4, atol=1e-1)


@pytest.mark.parametrize("R,C,yld", [(16384, 2560, 2560), (300, 72, 72), (256, 64, 192)])
def test_relu_bwd_colsum(hip, R, C, yld):
    """Fused ReLU backward + bias gradient: masked = dy * (y > 0), db = colsum(masked), vs torch;
    y may be a column slice of a wider buffer (row stride != C); -0.0 and +0.0 are masked."""
    dy = _rand(R, C, seed=50)
    ybuf = _rand(R, yld, seed=51)
    ybuf[0, :4] = torch.tensor([0.0, -0.0, 1e-30, -1e-30], dtype=torch.bfloat16)
    y = ybuf[:, :C]
    masked, db = hip.relu_bwd_colsum(dy, y, R, C)
    ref = dy.float() * (y.float() > 0).float()
    torch.testing.assert_close(masked.float(), ref, rtol=0, atol=0)
    torch.testing.assert_close(db, ref.sum(0), rtol=1e-4, atol=1e-2)
    # the bias-free form (flat full-chip grid, no column sums) gives the same masked gradient
    torch.testing.assert_close(hip.relu_bwd(dy, y, R, C).float(), ref, rtol=0, atol=0)


def test_ticket_reductions_rearm(hip):
    """Last-arriver reductions (sum_all, colsum) re-arm their tickets: repeated calls with
    different data and grid sizes stay exact, and sum_all writes bf16 directly."""
    for i, n in enumerate((1 << 22, 3 * (1 << 20) + 8, 4096, 1 << 22)):
        x = _rand(n, seed=100 + i)
        ref = x.float().sum()
        torch.testing.assert_close(hip.sum_all(x, torch.float32), ref, rtol=1e-3, atol=1e-1)
        got = hip.sum_all(x, torch.bfloat16)
        assert got.dtype == torch.bfloat16
        torch.testing.assert_close(got.float(), ref, rtol=1e-2, atol=1.0)
    for i, (R, C) in enumerate(((16384, 1536), (1000, 64), (16384, 640), (77, 8))):
        m = _rand(R, C, seed=200 + i)
        out = hip.colsum(m)
        torch.testing.assert_close(out, m.float().sum(0), rtol=1e-4, atol=5e-2)
        hip.colsum(m, out=out, accumulate=True)
        torch.testing.assert_close(out, 2 * m.float().sum(0), rtol=1e-4, atol=1e-1)
    row = _rand(320, seed=300)
    got = hip.colsum_ld(row, 1000, 320, 0)
    torch.testing.assert_close(got, row.float() * 1000, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("S,R,C,cb", [(8, 640, 1536, 512), (16, 512, 640, 640), (3, 40, 24, 8), (24, 512, 640, 640), (11, 640, 512, 512), (30, 64, 64, 64)])
def test_slab_reduce(hip, S, R, C, cb):
    slabs = _rand(S, R, C, dtype=torch.float32, seed=400 + S)
    nb = C // cb
    out = torch.empty((nb, R, cb), dtype=torch.float32, device=dev)
    hip.slab_reduce(slabs, out, cb, R * cb)
    ref = slabs.sum(0).reshape(R, nb, cb).permute(1, 0, 2)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-4)
    hip.slab_reduce(slabs, out, cb, R * cb, accumulate=True)
    torch.testing.assert_close(out, 2 * ref, rtol=1e-5, atol=2e-4)


@pytest.mark.parametrize("T,K,N,S", [(16384, 640, 2560, 5), (16384, 512, 640, 24), (4160, 256, 384, 4),
                                     (16384, 2560, 640, 5)])
@pytest.mark.parametrize("tile", [1282, 2563, 12856])
def test_gemm_slab_mode_uneven_splits(hip, T, K, N, S, tile):
    """Slab mode: split s of the token range writes slab s, the last split runs past T (zeros
    from the range check) -- the slabs sum to X^T dY, and each slab is its own token range."""
    assert hip.slab_count(T // 64, S) == S
    x, dy = _rand(T, K, seed=70), _rand(T, N, seed=71)
    slabs = torch.full((S, K, N), float("nan"), dtype=torch.float32, device=dev)
    hip.gemm(x, dy, slabs, K, N, T, K, N, N, False, False, sC=K * N, splitk=S, tile=tile, slabs=True)
    ref = x.float().t() @ dy.float()
    torch.testing.assert_close(slabs.sum(0), ref, rtol=2e-3, atol=2e-3 * ref.abs().max().item())
    kc = -(-(T // 64) // S) * 64
    last = x[kc * (S - 1):].float().t() @ dy[kc * (S - 1):].float()
    torch.testing.assert_close(slabs[S - 1], last, rtol=2e-3, atol=2e-3 * last.abs().max().item())


@pytest.mark.parametrize("T", [16384, 4096, 192])
def test_linear_weight_grad_slabs(hip, T):
    """dW of the fused QKV dense (3 kernels, one [T][1536] cotangent) and of a single dense with a
    broadcast-row cotangent, through the K-chunk slab GEMM + combine, vs fp32 torch."""
    x = _rand(T, 640, seed=11)
    ws = [(_rand(640, 512, dtype=torch.float32, seed=12 + i) * 0.05).requires_grad_() for i in range(3)]
    ys = hip.linear(x, ws, None, torch.bfloat16, False, torch.bfloat16)
    big = _rand(T, 1536, seed=20)
    for dys in ([big[:, 512 * i:512 * (i + 1)] for i in range(3)],      # column blocks: one batched GEMM
                [_rand(T, 512, seed=21 + i) for i in range(3)]):        # separate buffers
        grads = torch.autograd.grad(ys, ws, dys, retain_graph=True)
        for g, dy in zip(grads, dys):
            ref = x.float().t() @ dy.float()
            torch.testing.assert_close(g, ref, rtol=2e-3, atol=2e-3 * ref.abs().max().item())
    w = (_rand(512, 640, dtype=torch.float32, seed=30) * 0.05).requires_grad_()
    xo = _rand(T, 512, seed=31)
    (y,) = hip.linear(xo, [w], None, torch.bfloat16, False, torch.bfloat16)
    row = _rand(640, seed=32)
    (g,) = torch.autograd.grad([y], [w], [row.expand(T, 640)])
    ref = xo.float().sum(0)[:, None] * row.float()[None, :]
    torch.testing.assert_close(g, ref, rtol=2e-3, atol=2e-3 * ref.abs().max().item())


def test_sum_backward_broadcast_row(hip):
    x = _rand(8, 16, 96, seed=5).requires_grad_()
    s = hip.sum_all(x, torch.bfloat16)
    (g,) = torch.autograd.grad(s, [x], torch.tensor(0.25, dtype=torch.bfloat16, device=dev))
    assert g.shape == x.shape and g.stride()[:2] == (0, 0)
    torch.testing.assert_close(g.float(), torch.full(x.shape, 0.25, device=dev))


@pytest.mark.parametrize("S0,S1,tile", [(4, 12, 1282), (8, 24, 1282), (4, 5, 1282), (3, 3, 12884), (2, 6, 12883)])
def test_gemm_group_two_slab_gemms_bit_exact(hip, S0, S1, tile):
    """Two weight-gradient slab GEMMs (the bench's dW_qkv batch of 3 and dW_o) launched as one
    grouped grid write exactly what two separate launches write; a group of one GEMM, and two of
    different tiles, launch one by one."""
    dev = "cuda"
    torch.manual_seed(0)
    T = 2048
    x = torch.randn(T, 640, device=dev).bfloat16()
    dq = [torch.randn(T, 512, device=dev).bfloat16() for _ in range(3)]
    h = torch.randn(T, 512, device=dev).bfloat16()
    dy = torch.randn(T, 640, device=dev).bfloat16()
    nkt = T // 64
    s0, s1 = hip.slab_count(nkt, S0), hip.slab_count(nkt, S1)

    def run(group, tile1=tile):
        sl0 = torch.full((s0, 3, 640, 512), float("nan"), device=dev)
        sl1 = torch.full((s1, 512, 640), float("nan"), device=dev)
        if group:
            hip.gemm_group_begin()
        hip.gemm(x, dq[0], sl0, 640, 512, T, 640, 512, 512, False, False, batch=3, sA=0, sC=640 * 512,
                 splitk=s0, tile=tile, slabs=True, b_list=dq)
        hip.gemm(h, dy, sl1, 512, 640, T, 512, 640, 640, False, False, sC=512 * 640, splitk=s1, tile=tile1,
                 slabs=True)
        if group:
            hip.gemm_group_end(sl0)
        torch.cuda.synchronize()
        return sl0, sl1

    r0, r1 = run(False)
    g0, g1 = run(True)
    assert torch.equal(r0, g0) and torch.equal(r1, g1)
    # against an fp32 reference of the slab sums
    ref1 = h.float().t() @ dy.float()
    torch.testing.assert_close(g1.sum(0), ref1, rtol=2e-3, atol=2e-2)
    m0, m1 = run(True, tile1=1284)   # different instances: launched one by one
    assert torch.equal(r0, m0)
    torch.testing.assert_close(m1.sum(0), ref1, rtol=2e-3, atol=2e-2)
    hip.gemm_group_begin()
    hip.gemm_group_end(x)             # empty group: nothing launched


def test_adam_multi_folded_step_increment(hip):
    """increment_step advances the device count by one per call (the one-lane launch) and the bias
    corrections use the new count."""
    ws = [torch.randn(64 * 7, 130, device=dev) for _ in range(40)]  # > 32 tensors: two launches
    gs = [torch.randn_like(w) for w in ws]
    ms = [torch.zeros_like(w) for w in ws]
    vs = [torch.zeros_like(w) for w in ws]
    refs = [w.clone().requires_grad_() for w in ws]
    opt = torch.optim.Adam(refs, lr=1e-3)
    step = torch.zeros((), dtype=torch.int32, device=dev)
    for k in range(3):
        hip.adam_multi(list(zip(ws, gs, ms, vs)), step, 1e-3, 0.9, 0.999, 1e-8, 0.0, increment_step=True)
        assert int(step) == k + 1
        for r, g in zip(refs, gs):
            r.grad = g.clone()
        opt.step()
    for w, r in zip(ws, refs):
        torch.testing.assert_close(w, r.detach(), rtol=1e-5, atol=1e-6)


# ----------------------------------------------------------------------------- MX-fp8
def test_fp8_quantization_matches_reference(hip):
    from learning_jax_sharding_amd.ops import fp8 as F
    x = _rand(300, 256, dtype=torch.float32, seed=40) * 3
    x[5, :32] = 0.0                       # all-zero block
    x[7, 40] = 1e4                        # outlier block
    q, s = F.quant_rows(x)
    qr, er = F.quantize_mx_ref(x.cpu())
    assert torch.equal(s.cpu().long(), (er + 127).long())
    assert torch.equal(q.cpu(), qr.view(torch.uint8))
    qb, sb = F.quant_rows(x.bfloat16())
    qr2, er2 = F.quantize_mx_ref(x.bfloat16().cpu())
    assert torch.equal(qb.cpu(), qr2.view(torch.uint8)) and torch.equal(sb.cpu().long(), (er2 + 127).long())
    w = _rand(256, 136, dtype=torch.float32, seed=41) * 0.05
    qc, sc = F.quant_cols(w)
    qr3, er3 = F.quantize_mx_ref(w.t().contiguous().cpu())
    assert torch.equal(qc.cpu(), qr3.view(torch.uint8)) and torch.equal(sc.cpu().long(), (er3 + 127).long())
    # the LDS-tiled bf16 path (K % 128, N % 64), incl. a row-strided view
    xb = (_rand(1024, 704, dtype=torch.float32, seed=42) * 2).bfloat16()
    xb[64:96, 5] = 0
    for src in (xb[:, :640], xb[:, 64:]):
        qt, st = F.quant_cols(src)
        qr4, er4 = F.quantize_mx_ref(src.t().contiguous().cpu())
        assert torch.equal(qt.cpu(), qr4.view(torch.uint8)) and torch.equal(st.cpu().long(), (er4 + 127).long())
        # one pass, both layouts
        (q1, s1), (q2, s2) = F._quant_both(src)
        qr5, sr5 = F.quant_rows(src)
        assert torch.equal(q1, qr5) and torch.equal(s1, sr5) and torch.equal(q2, qt) and torch.equal(s2, st)


def test_fp8_quantization_f32_emits_bf16_copy(hip):
    """The f32-input forms round x to bf16 inside the quantization pass and write that copy: bit-
    identical to a cast pass followed by the bf16 quantization (the MX layer's input cast fused)."""
    from learning_jax_sharding_amd.ops import fp8 as F
    x = _rand(1024, 704, dtype=torch.float32, seed=45) * 2
    x[64:96, 5] = 0
    x[3, 7] = 3e4
    for src in (x[:, :640], x[:, 64:].contiguous()):
        ref = src.bfloat16()
        if src.is_contiguous():
            xb = torch.full(src.shape, 7.0, dtype=torch.bfloat16, device=dev)
            (q1, s1), (q2, s2) = F._quant_both(src, xb)
            (r1, t1), (r2, t2) = F._quant_both(ref)
            assert torch.equal(xb, ref)
            assert torch.equal(q1, r1) and torch.equal(s1, t1) and torch.equal(q2, r2) and torch.equal(s2, t2)
        else:
            with pytest.raises(AssertionError):
                F._quant_both(src, None)
        xr = torch.full((src.shape[0], src.shape[1]), 7.0, dtype=torch.bfloat16, device=dev)
        qa, sa = F.quant_rows(src, xb=xr)
        qb, sb = F.quant_rows(src)
        assert torch.equal(xr, ref) and torch.equal(qa, qb) and torch.equal(sa, sb)


def test_fp8_ff_block_f32_input_has_no_cast_pass(hip):
    """An f32 input to the MX FF block: the output and grads equal the bf16-input block's (the
    fused cast is the same rounding), and no standalone f32->bf16 cast kernel runs."""
    from learning_jax_sharding_amd.ops import fp8 as F
    from learning_jax_sharding_amd.ops import hip as H
    x = _rand(256, 128, dtype=torch.float32, seed=46)
    wi = (_rand(128, 512, dtype=torch.float32, seed=47) * 0.05).requires_grad_()
    wo = (_rand(512, 128, dtype=torch.float32, seed=48) * 0.05).requires_grad_()
    calls = []
    orig = H._cast_raw
    H._cast_raw = lambda *a, **k: (calls.append(1), orig(*a, **k))[1]
    try:
        y = F._FFBlockFp8.apply(x, wi, wo, x)
    finally:
        H._cast_raw = orig
    assert not calls
    wi2 = wi.detach().clone().requires_grad_()
    wo2 = wo.detach().clone().requires_grad_()
    xb = x.bfloat16()
    y2 = F._FFBlockFp8.apply(xb, wi2, wo2, xb)
    assert torch.equal(y, y2)
    y.float().sum().backward()
    y2.float().sum().backward()
    assert torch.equal(wi.grad, wi2.grad) and torch.equal(wo.grad, wo2.grad)


@pytest.mark.parametrize("tile", [1282, 1283, 2562, 2563])
@pytest.mark.parametrize("M,N,K", [(128, 128, 128), (300, 136, 256), (1024, 2560, 640), (512, 640, 2560)])
@pytest.mark.parametrize("bias,relu,out_f32", [(False, False, True), (True, True, False)])
def test_fp8_gemm_matches_emulation(hip, M, N, K, bias, relu, out_f32, tile):
    from learning_jax_sharding_amd.ops import fp8 as F
    x = _rand(M, K, dtype=torch.float32, seed=42)
    w = _rand(K, N, dtype=torch.float32, seed=43) * 0.05
    b = _rand(N, dtype=torch.float32, seed=44) if bias else None
    qa, sa = F.quant_rows(x)
    qb, sb = F.quant_cols(w)
    out = torch.empty((M, N), dtype=torch.float32 if out_f32 else torch.bfloat16, device=dev)
    F.gemm_mx(qa, sa, qb, sb, M, N, K, out, b, relu, tile=tile)
    ref = F.mx_linear_ref(x.cpu(), w.cpu(), None if b is None else b.cpu(), relu, out.dtype)
    tol = 1e-3 if out_f32 else 2e-2
    torch.testing.assert_close(out.float().cpu(), ref.float(), rtol=tol, atol=tol * 4)


@pytest.mark.parametrize("tile", [1282, 2563])
@pytest.mark.parametrize("mode", ["add", "mask", None])
def test_fp8_gemm_epilogue_residual_mask_and_quantized_copy(hip, tile, mode):
    """MX-fp8 GEMM epilogue: residual add / ReLU mask on a bf16 operand (bit-exact with the
    unfused ops on the plain output) and the MX-fp8 copy of the output (== quant_rows of it)."""
    from learning_jax_sharding_amd.ops import fp8 as F
    M, N, K = 1024, 640, 512
    qa, sa = F.quant_rows(_rand(M, K, dtype=torch.float32, seed=48))
    qb, sb = F.quant_cols(_rand(K, N, dtype=torch.float32, seed=49) * 0.05)
    plain = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
    F.gemm_mx(qa, sa, qb, sb, M, N, K, plain, tile=tile)
    R = _rand(M, N, seed=50)
    if mode == "mask":
        R = torch.relu(R)
    out = torch.empty_like(plain)
    q = torch.empty((M, N), dtype=torch.uint8, device=dev)
    sc = torch.empty((M, N // 32), dtype=torch.uint8, device=dev)
    F.gemm_mx(qa, sa, qb, sb, M, N, K, out, res=R if mode else None, res_mode=mode or "add", qout=(q, sc), tile=tile)
    torch.cuda.synchronize()
    # masked elements are +0 (as the bf16 GEMM's mask and relu_bwd write them)
    ref = plain + R if mode == "add" else (torch.where(R > 0, plain, torch.zeros_like(plain)) if mode == "mask"
                                           else plain)
    assert torch.equal(out, ref)
    q2, s2 = F.quant_rows(ref)
    assert torch.equal(q, q2) and torch.equal(sc, s2)


def test_fp8_linear_autograd(hip):
    from learning_jax_sharding_amd.ops import fp8 as F
    x = _rand(256, 512, dtype=torch.bfloat16, seed=45).requires_grad_()
    w = (_rand(512, 384, dtype=torch.float32, seed=46) * 0.05).requires_grad_()
    b = torch.zeros(384, device=dev, requires_grad=True)
    y = F.linear_fp8(x, w, b, True, torch.bfloat16)
    g = _rand(256, 384, seed=47)
    (y.float() * g.float()).sum().backward()
    ref = F.mx_linear_ref(x.detach().cpu(), w.detach().cpu(), b.detach().cpu(), True, torch.bfloat16)
    torch.testing.assert_close(y.float().cpu(), ref.float(), rtol=2e-2, atol=3e-2)
    mask = (y > 0).float()
    gm = g.float() * mask
    torch.testing.assert_close(w.grad, x.detach().float().t() @ gm, rtol=3e-2, atol=3e-1)
    torch.testing.assert_close(x.grad.float(), gm @ w.detach().bfloat16().float().t(), rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(b.grad, gm.sum(0), rtol=1e-2, atol=1e-1)


def test_native_runtime_device_info_and_single_member_comm(hip):
    """Native runtime library: device properties and an ncclCommInitAll communicator (a
    1-member communicator on a one-GPU box; multi-GPU groups use the same calls)."""
    from learning_jax_sharding_amd.comm import native
    info = native.device_info(0)
    assert info["cus"] >= 1 and info["wavefront"] == 64 and info["hbm_bytes"] > 0
    nat = native.NativeRccl()
    t = torch.arange(1024, dtype=torch.float32, device=dev)
    nat.all_reduce([t])
    torch.cuda.synchronize()
    torch.testing.assert_close(t, torch.arange(1024, dtype=torch.float32, device=dev))
    g = nat.all_gather([t[:16].contiguous()])
    torch.cuda.synchronize()
    assert g[0].shape == (1, 16)
    nat.close()
    maps = open(f"/proc/{__import__('os').getpid()}/maps").read()
    assert "libljs_runtime.so" in maps


@pytest.mark.parametrize("T,M,Fd,bcast,self_res", [(2048, 640, 2560, False, False), (1024, 256, 512, True, False),
                                                   (2048, 640, 2560, False, True), (1024, 256, 512, True, True)])
def test_fp8_ff_block_matches_emulation(hip, T, M, Fd, bcast, self_res):
    """Fused MX-fp8 FF block on the GPU (fp8 forward + fp8 dX GEMMs, epilogue-quantized
    operands, fused residual / ReLU mask, broadcast dY read as one row, the skip gradient of a
    residual that is x folded into dX's epilogue) == its host emulation, to f32 summation order."""
    from learning_jax_sharding_amd.ops import fp8 as F
    x = _rand(T, M, seed=60).requires_grad_()
    wi = (_rand(M, Fd, dtype=torch.float32, seed=61) * 0.05).requires_grad_()
    wo = (_rand(Fd, M, dtype=torch.float32, seed=62) * 0.03).requires_grad_()
    res = x if self_res else _rand(T, M, seed=63).requires_grad_()
    y = F.ff_block_local(x, wi, wo, res)
    cot = torch.full((), 0.5, dtype=torch.bfloat16, device=dev).expand(T, M) if bcast else _rand(T, M, seed=64)
    y.backward(cot)
    xc, wic, woc = (t.detach().cpu().requires_grad_() for t in (x, wi, wo))
    rc = xc if self_res else res.detach().cpu().requires_grad_()
    yc = F.ff_block_local(xc, wic, woc, rc)
    yc.backward(cot.cpu())
    # an f32 summation-order difference can move a value across a bf16 / e4m3 rounding boundary
    # (a handful of elements of the 1.3 M)
    d = (y.float().cpu() - yc.float()).abs()
    assert (d > 2e-2 + 2e-2 * yc.float().abs()).float().mean().item() < 1e-4
    assert (d.norm() / yc.float().norm()).item() < 5e-3   # ~1 bf16 ulp where sums differ
    for got, want in ((x.grad, xc.grad), (wi.grad, wic.grad), (wo.grad, woc.grad), (res.grad, rc.grad)):
        err = ((got.float().cpu() - want.float()).norm() / want.float().norm().clamp(min=1e-6)).item()
        assert err < 2e-2, err


@pytest.mark.parametrize("rdt", [torch.float32, torch.bfloat16])
def test_linear_seq_major_rows_batch_major_residual(hip, rdt):
    """Seq-major x with a batch-major residual (the 2-D mesh's out projection + the layer's skip):
    the residual is transposed to the row order and rounded to bf16 in one pass - y bit-equal to
    the batch-major run (the epilogue rounds the residual to bf16 before the add either way)."""
    from learning_jax_sharding_amd.ops import linear as L
    B, S, K, N = 8, 256, 512, 320
    base = _rand(S, B, K, seed=80)
    w = _rand(K, N, dtype=torch.float32, seed=81) * 0.05
    r = _rand(B, S, N, dtype=rdt, seed=82)
    ys = {}
    for seq_major in (True, False):
        x = base.permute(1, 0, 2) if seq_major else base.permute(1, 0, 2).contiguous()
        ys[seq_major] = L.linear(x, [w], None, False, torch.bfloat16, residual=r)[0]
    assert ys[True].stride() == (N, B * N, 1)   # rows in x's (seq-major) storage order
    assert torch.equal(ys[True], ys[False])


@pytest.mark.parametrize("bcast", [False, True])
def test_ff_block_bf16_seq_major_rows(hip, bcast):
    """The bf16 fused FF block (residual x) on a seq-major activation runs in its storage row
    order: y and dX bit-equal to the batch-major run and laid out like x; the weight gradients
    (split-K token sums in another order) to f32 summation order."""
    from learning_jax_sharding_amd.ops import linear as L
    B, S, M, Fd = 8, 128, 256, 512
    base = _rand(S, B, M, seed=90)
    wi0 = _rand(M, Fd, dtype=torch.float32, seed=91) * 0.05
    wo0 = _rand(Fd, M, dtype=torch.float32, seed=92) * 0.03
    cot = torch.full((), 0.5, dtype=torch.bfloat16, device=dev).expand(B, S, M) if bcast else \
        _rand(S, B, M, seed=93).permute(1, 0, 2)
    res = {}
    for seq_major in (True, False):
        x = (base.permute(1, 0, 2) if seq_major else base.permute(1, 0, 2).contiguous()).detach().requires_grad_()
        wi, wo = wi0.clone().requires_grad_(), wo0.clone().requires_grad_()
        y = L.ff_block(x, wi, wo, True)
        if seq_major:
            assert y.stride() == x.stride(), (y.stride(), x.stride())
        y.backward(cot)
        res[seq_major] = (y.detach(), x.grad, wi.grad, wo.grad)
    assert torch.equal(res[True][0], res[False][0])
    assert torch.equal(res[True][1], res[False][1])
    for a, b_ in zip(res[True][2:], res[False][2:]):
        torch.testing.assert_close(a, b_, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("bcast", [False, True])
def test_fp8_ff_block_seq_major_rows(hip, bcast):
    """A seq-major activation (batch, seq, M) stored [seq][batch][M] - the 2-D mesh's out
    projection output - runs the fused MX-fp8 FF block in its storage row order without a copy:
    y and dX (per-token rows, the residual x folded in) bit-equal to the batch-major run and laid
    out like x; the weight gradients sum the tokens in another order AND block them differently
    for their MX operands (32 consecutive storage rows share a scale), so they agree to the MX
    quantization noise of two groupings (~3 % relative norm each), not bit for bit."""
    from learning_jax_sharding_amd.ops import fp8 as F
    B, S, M, Fd = 8, 128, 256, 512
    base = _rand(S, B, M, seed=70)
    wi0 = _rand(M, Fd, dtype=torch.float32, seed=71) * 0.05
    wo0 = _rand(Fd, M, dtype=torch.float32, seed=72) * 0.03
    cot = torch.full((), 0.5, dtype=torch.bfloat16, device=dev).expand(B, S, M) if bcast else \
        _rand(S, B, M, seed=73).permute(1, 0, 2)
    res = {}
    for seq_major in (True, False):
        x = (base.permute(1, 0, 2) if seq_major else base.permute(1, 0, 2).contiguous()).detach().requires_grad_()
        wi, wo = wi0.clone().requires_grad_(), wo0.clone().requires_grad_()
        y = F.ff_block_local(x, wi, wo, x)
        if seq_major:
            assert y.stride() == x.stride(), (y.stride(), x.stride())
        y.backward(cot)
        res[seq_major] = (y.detach(), x.grad, wi.grad, wo.grad)
    assert torch.equal(res[True][0], res[False][0])
    assert torch.equal(res[True][1], res[False][1])
    for a, b_ in zip(res[True][2:], res[False][2:]):
        err = ((a.float() - b_.float()).norm() / b_.float().norm().clamp(min=1e-6)).item()
        assert err < 6e-2, err


def test_fp8_transformer_layer_trains(gpu_devices):
    """TransformerLayer(fp8=True) takes the fused fp8 FF block and its train step runs."""
    gpu_devices(1)
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd.models import TransformerLayer
    from learning_jax_sharding_amd.spmd import plan as _plan
    model = TransformerLayer(640, heads=8, dim_head=64, ff_dim=2560, fp8=True)
    x = ljs.random.normal(ljs.random.PRNGKey(0), (2, 256, 640))
    params = model.init(ljs.random.PRNGKey(1), x)["params"]
    with _plan.record_plan() as rec:
        val, g = ljs.value_and_grad(lambda p: model.apply({"params": p}, x).sum())(params)
    torch.cuda.synchronize()
    assert any(st.kind == "ff_block" for st in rec.steps)
    leaves = ljs.tree_util.tree_leaves(ljs.nn.unbox(g))
    assert all(torch.isfinite(l.to_torch()).all() for l in leaves)


@pytest.mark.parametrize("shape,dim,n", [((8, 256, 640), 0, 4), ((8, 256, 640), 1, 2), ((4, 6, 10), 2, 5),
                                         ((3, 7), 1, 7), ((16,), 0, 8), ((2, 8, 3), 1, 4)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32, torch.uint8])
def test_collective_pack_unpack(hip, shape, dim, n, dtype):
    """HIP pack / unpack around collectives == the torch movedim / index / cat formulation
    (rank permutations, 16 / 4 / 1-byte units)."""
    g = torch.Generator(device="cpu").manual_seed(7)
    x = (torch.randn(shape, generator=g) * 50).to(dtype).to(dev)
    perm = list(range(n))[::-1] if n > 1 else [0]
    s = shape[dim] // n
    ref = x.reshape(shape[:dim] + (n, s) + shape[dim + 1:]).movedim(dim, 0)
    assert torch.equal(hip.rank_major(x, dim, n), ref.contiguous())
    assert torch.equal(hip.rank_major(x, dim, n, perm), ref[perm].contiguous())
    buf = ref.contiguous()
    assert torch.equal(hip.from_rank_major(buf, dim), x)
    assert torch.equal(hip.from_rank_major(buf[perm].contiguous(), dim, perm), x)
    parts = [t.contiguous() for t in x.chunk(n, dim)]
    assert torch.equal(hip.concat_parts(parts, dim), torch.cat(parts, dim))


def test_fp8_gemm_transposed_copy_splitk_bcast_and_fp8_mask(hip):
    """MX GEMM options of the fp8 FF block: the transposed MX copy == quant_cols of the bf16
    output (bit-exact), split-K slabs sum to the unsplit f32 result, a broadcast B row == the
    materialised rows, and a ReLU mask read from e4m3 bytes == the mask of their bf16 values."""
    from learning_jax_sharding_amd.ops import fp8 as F
    T, N, K = 1024, 640, 512
    x, w = _rand(T, K, seed=80), _rand(N, K, seed=81)
    qa, sa = F.quant_rows(x)
    qb, sb = F.quant_rows(w)
    c = torch.empty(T, N, dtype=torch.bfloat16, device=dev)
    F.gemm_mx(qa, sa, qb, sb, T, N, K, c, relu=True)
    qt = torch.empty(N, T, dtype=torch.uint8, device=dev)
    st = torch.empty(N, T // 32, dtype=torch.uint8, device=dev)
    q = torch.empty(T, N, dtype=torch.uint8, device=dev)
    s = torch.empty(T, N // 32, dtype=torch.uint8, device=dev)
    F.gemm_mx(qa, sa, qb, sb, T, N, K, None, relu=True, qout=(q, s), qtout=(qt, st))
    qt_ref, st_ref = F.quant_cols(c)
    assert torch.equal(qt, qt_ref) and torch.equal(st, st_ref)
    q_ref, s_ref = F.quant_rows(c)
    assert torch.equal(q, q_ref) and torch.equal(s, s_ref)
    # split-K (uneven last split: 4 K-tiles over 3 splits)
    full = torch.empty(T, N, device=dev)
    F.gemm_mx(qa, sa, qb, sb, T, N, K, full)
    assert hip.slab_count(K // 128, 3) == 2   # 4 K-tiles: 3 requested -> 2 x 2
    slabs = torch.empty(2, T, N, device=dev)
    F.gemm_mx(qa, sa, qb, sb, T, N, K, slabs, nsplit=2)
    torch.testing.assert_close(slabs.sum(0), full, rtol=1e-5, atol=1e-4)
    # broadcast B row
    wb = _rand(1, K, seed=82)
    qbr, sbr = F.quant_rows(wb)
    o1 = torch.empty(T, N, device=dev)
    o2 = torch.empty(T, N, device=dev)
    F.gemm_mx(qa, sa, qbr, sbr, T, N, K, o1, b_bcast=True)
    F.gemm_mx(qa, sa, qbr.expand(N, K).contiguous(), sbr.expand(N, K // 32).contiguous(), T, N, K, o2)
    assert torch.equal(o1, o2)
    # ReLU mask from e4m3 bytes (q of the ReLU output) == mask from their dequantized bf16 values
    vals = q.view(torch.float8_e4m3fn).float().reshape(T, N // 32, 32)
    dq = (vals * torch.ldexp(torch.ones_like(vals[..., :1]), s.int()[..., None] - 127)).reshape(T, N).bfloat16()
    m1 = torch.empty(T, N, dtype=torch.bfloat16, device=dev)
    m2 = torch.empty(T, N, dtype=torch.bfloat16, device=dev)
    F.gemm_mx(qa, sa, qb, sb, T, N, K, m1, res=q, res_mode="mask")
    F.gemm_mx(qa, sa, qb, sb, T, N, K, m2, res=dq, res_mode="mask")
    assert torch.equal(m1, m2)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("sk", [128, 512])
def test_attention_fwd_inkernel_lse_merge(causal, sk):
    """Ring attention's forward: key blocks merged by log-sum-exp in the kernel epilogue (f32
    running output + lse, modes 1 / 2 / 3) == one attention over all keys (f32 oracle), including
    a causal block that is fully masked for some rows (+inf lse)."""
    from learning_jax_sharding_amd.ops import hip, kernels as K
    torch.manual_seed(0)
    B, Sq, H = 2, 128, 4
    nblk = 3
    q = torch.randn(B, Sq, H, 64, device="cuda").bfloat16()
    k = torch.randn(B, nblk * sk, H, 64, device="cuda").bfloat16()
    v = torch.randn(B, nblk * sk, H, 64, device="cuda").bfloat16()
    q_off = sk if causal else 0     # causal: queries aligned with block 1 -> block 2 fully masked (+inf lse)
    ref = K.attention_reference(q, k, v, 0.125, causal, q_off).float()
    state = [None, None]
    out = None
    for i in range(nblk):
        kb, vb = k[:, i * sk:(i + 1) * sk], v[:, i * sk:(i + 1) * sk]
        out = K.attention_fwd_merge(q, kb, vb, 0.125, causal, q_off - i * sk, state, last=i == nblk - 1)
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.float().cpu().numpy(), ref.cpu().numpy(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("shape", [(640, 1920), (64, 8), (100, 264), (3, 8)])
def test_transpose_bf16_and_swap01(hip, shape):
    """Vectorised LDS transpose and the (a, b, c) -> (b, a, c) swap == torch (bit-exact, ragged
    edges included)."""
    x = torch.randn(shape, device="cuda").bfloat16()
    assert torch.equal(hip.transpose_bf16(x), x.t().contiguous())
    y = torch.randn(4, shape[0], 8, device="cuda").bfloat16()
    assert torch.equal(hip.swap01_bf16(y), y.transpose(0, 1).contiguous())
    z = torch.randn(3, shape[0], 24, device="cuda")       # f32 in: rounded in the same pass
    assert torch.equal(hip.swap01_bf16(z), z.transpose(0, 1).contiguous().bfloat16())


@pytest.mark.parametrize("n", [1, 2, 4, 7, 100])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_sum_n(hip, n, dtype):
    """One-launch n-way sum (f32 accumulation, pointers by value) == the f32 torch sum."""
    xs = [torch.randn(1000 + 8 * n, 24, device="cuda").to(dtype) for _ in range(n)]
    ref = torch.stack([x.float() for x in xs]).sum(0)
    out = hip.sum_n(xs)
    torch.cuda.synchronize()
    tol = 0 if dtype == torch.float32 and n <= 2 else 1e-2
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("R,C", [(1, 5), (3, 64), (64, 640), (37, 1000), (200, 130)])
def test_rows_sum(hip, R, C):
    """Short-matrix row sum (the fused column-sum partials) == the f32 torch sum; a strided view too."""
    base = torch.randn(R, C + 8, device="cuda")
    x = base[:, :C]
    out = hip.rows_sum(x)
    torch.cuda.synchronize()
    torch.testing.assert_close(out, x.double().sum(0).float(), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("tile", [256256, 256128, 256160, 128320, 128256, 128128, 128160, 3128128, 3128160, 3128256, 3256128])
@pytest.mark.parametrize("mode", ["qboth", "qmask8", "res_bias", "f32split"])
def test_fp8_gemm_8wave_tiles_match_4wave(hip, tile, mode):
    """The 8-wave large-tile MX GEMM runs the same MFMA sequence per output element as the 4-wave
    128x128 kernel: every output (bf16 rows, row-blocked and transposed MX copies, f32 split-K
    slabs) must be bit-identical, edges included (M, N not multiples of the tile)."""
    from learning_jax_sharding_amd.ops import fp8 as F
    g = torch.Generator(device="cpu").manual_seed(tile % 997)
    T, N, K = 1056, 640, 512
    x = torch.randn(T, K, generator=g).bfloat16().to(dev)
    w = torch.randn(N, K, generator=g).bfloat16().to(dev)
    qa, sa = F.quant_rows(x)
    qb, sb = F.quant_rows(w)
    r = torch.randn(T, N, generator=g).bfloat16().to(dev)
    r8, _ = F.quant_rows(r)
    bias = torch.randn(N, generator=g).to(dev)

    def run(t):
        if mode in ("qboth", "qmask8"):
            o = [torch.full((T, N), 7, dtype=torch.uint8, device=dev), torch.zeros((T, N // 32), dtype=torch.uint8, device=dev),
                 torch.full((N, T), 7, dtype=torch.uint8, device=dev), torch.zeros((N, T // 32), dtype=torch.uint8, device=dev)]
            if mode == "qboth":
                F.gemm_mx(qa, sa, qb, sb, T, N, K, None, relu=True, qout=(o[0], o[1]), qtout=(o[2], o[3]), tile=t)
            else:
                F.gemm_mx(qa, sa, qb, sb, T, N, K, None, res=r8, res_mode="mask", qout=(o[0], o[1]),
                          qtout=(o[2], o[3]), tile=t)
            return o
        if mode == "f32split":
            c = torch.zeros((2, T, N), dtype=torch.float32, device=dev)
            F.gemm_mx(qa, sa, qb, sb, T, N, K, c, nsplit=2, tile=t)
            return [c]
        c = torch.zeros((T, N), dtype=torch.bfloat16, device=dev)
        F.gemm_mx(qa, sa, qb, sb, T, N, K, c, bias=bias, relu=True, res=r, tile=t)
        return [c]

    ref, out = run(1282), run(tile)
    torch.cuda.synchronize()
    for a, b in zip(ref, out):
        assert torch.equal(a, b)


@pytest.mark.parametrize("tile", [1282, 12883, 12884, 2563])
def test_gemm_slab_mode_batched_weights(hip, tile):
    """Slab mode over a batch of weight-major cotangents (shared X, dY_i at stride T*N): slab
    [s][i] = split s of weight i, bit-identical to the one-weight launches."""
    T, K, N, nw = 4096, 640, 512, 3
    S = 4
    assert hip.slab_count(T // 64, S) == S
    x = _rand(T, K, seed=80)
    dys = _rand(nw * T, N, seed=81).view(nw, T, N)
    slabs = torch.full((S, nw, K, N), float("nan"), dtype=torch.float32, device=dev)
    hip.gemm(x, dys, slabs, K, N, T, K, N, N, False, False, batch=nw, sA=0, sB=T * N, sC=K * N, splitk=S,
             tile=tile, slabs=True)
    # the same batch from separate B tensors (per-batch pointers)
    sep = [dys[i].clone() for i in range(nw)]
    slabs2 = torch.full((S, nw, K, N), float("nan"), dtype=torch.float32, device=dev)
    hip.gemm(x, sep[0], slabs2, K, N, T, K, N, N, False, False, batch=nw, sA=0, sC=K * N, splitk=S,
             tile=tile, slabs=True, b_list=sep)
    for i in range(nw):
        one = torch.full((S, K, N), float("nan"), dtype=torch.float32, device=dev)
        hip.gemm(x, dys[i], one, K, N, T, K, N, N, False, False, sC=K * N, splitk=S, tile=tile, slabs=True)
        assert torch.equal(slabs[:, i], one)
        assert torch.equal(slabs2[:, i], one)


@pytest.mark.parametrize("tile", [256160, 128160, 256256])
def test_fp8_gemm_fused_column_sums(hip, tile):
    """The 8-wave MX GEMM's epilogue column sums (per row tile, of the bf16 output including the
    residual add) == the f32 column sums of the output it wrote."""
    from learning_jax_sharding_amd.ops import fp8 as F
    g = torch.Generator(device="cpu").manual_seed(5)
    T, N, K = 1056, 640, 512
    qa, sa = F.quant_rows(torch.randn(T, K, generator=g).bfloat16().to(dev))
    qb, sb = F.quant_rows(torch.randn(N, K, generator=g).bfloat16().to(dev))
    r = torch.randn(T, N, generator=g).bfloat16().to(dev)
    c = torch.empty((T, N), dtype=torch.bfloat16, device=dev)
    bm = tile // 1000
    cs = torch.full((-(-T // bm), N), float("nan"), dtype=torch.float32, device=dev)
    F.gemm_mx(qa, sa, qb, sb, T, N, K, c, res=r, tile=tile, colsum=cs)
    torch.cuda.synchronize()
    ref = c.float().sum(0)
    torch.testing.assert_close(cs.sum(0), ref, rtol=1e-4, atol=1e-3 * ref.abs().max().item())
    sums = F._lazy_rows_sum(cs)()
    torch.testing.assert_close(sums, ref, rtol=1e-4, atol=1e-3 * ref.abs().max().item())


def test_fp8_transformer_layer_large_tiles_and_fused_colsum(gpu_devices):
    """At 4096 tokens the fp8 FF block's N=640 GEMMs take the 8-wave tiles and its dX GEMM writes
    the column sums the attention out-projection's bias gradient reads: that bias gradient ==
    the column sums of the same step with the fused sums off (fp8._FUSED_COLSUM = False), and
    every gradient is finite."""
    gpu_devices(1)
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd.models import TransformerLayer
    from learning_jax_sharding_amd.ops import fp8 as F
    model = TransformerLayer(640, heads=8, dim_head=64, ff_dim=1024, fp8=True)
    x = ljs.random.normal(ljs.random.PRNGKey(0), (16, 256, 640))
    params = model.init(ljs.random.PRNGKey(1), x)["params"]

    def grads():
        _, g = ljs.value_and_grad(lambda p: model.apply({"params": p}, x).sum())(params)
        torch.cuda.synchronize()
        return {"/".join(map(str, k)): v.to_torch().float().cpu()
                for k, v in ljs.tree_util.tree_flatten_with_path(ljs.nn.unbox(g))[0]} \
            if hasattr(ljs.tree_util, "tree_flatten_with_path") else \
            [l.to_torch().float().cpu() for l in ljs.tree_util.tree_leaves(ljs.nn.unbox(g))]

    assert F._auto_tile(4096, 640, 1024, 64, 1) >= 10000
    g1 = grads()
    old = F._FUSED_COLSUM
    F._FUSED_COLSUM = False
    try:
        g0 = grads()
    finally:
        F._FUSED_COLSUM = old
    items = g1.items() if isinstance(g1, dict) else enumerate(g1)
    for k, a in items:
        b = g0[k]
        assert torch.isfinite(a).all(), k
        torch.testing.assert_close(a, b, rtol=2e-3, atol=2e-3 * max(1.0, b.abs().max().item()))


@pytest.mark.parametrize("T,K,N,tile,S", [(16384, 640, 1536, 1282, 8), (16384, 512, 640, 1282, 24),
                                          (4096, 192, 328, 1282, 4), (8192, 640, 1536, 2563, 4)])
def test_slab_gemm_staged_epilogue_bit_exact(hip, T, K, N, tile, S):
    """Weight-gradient slab GEMMs: the last item's f32 tile through LDS as whole rows
    (kSlabVst) == the per-lane 16-byte stores, bit for bit (ragged M / N included)."""
    x = _rand(T, K, seed=21)
    dy = _rand(T, N, seed=22)
    assert hip.slab_count(T // 64, S) == S
    outs = []
    for vst in (True, False):
        hip._SLAB_VST = vst
        slabs = torch.full((S, K, N), float("nan"), dtype=torch.float32, device=dev)
        hip.gemm(x, dy, slabs, K, N, T, K, N, N, False, False, sC=K * N, splitk=S, tile=tile, slabs=True)
        outs.append(slabs)
    hip._SLAB_VST = True
    assert torch.equal(outs[0], outs[1])
    ref = (x.float().t() @ dy.float())
    torch.testing.assert_close(outs[0].sum(0), ref, rtol=2e-2, atol=2e-1)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_dropout_kernel_matches_host_philox_mask(hip, dtype):
    """The HIP dropout keeps element i iff the Philox uniform of its GLOBAL index is < keep (the
    host path's random.uniform draw, bit for bit); a shard's region selects its indices; the
    backward recomputes the same mask."""
    from learning_jax_sharding_amd import random as R
    shape = (4, 64, 96)
    key = R.PRNGKey(3)
    keep = 0.7
    full = torch.randn(shape).to(dtype)
    idx = np.arange(int(np.prod(shape)), dtype=np.uint64)
    u = torch.from_numpy(R._dist_np(idx, key, "uniform", 0.0, 1.0).astype(np.float32)).view(shape)
    ref = torch.where(u < keep, (full.float() / keep).to(dtype), torch.zeros((), dtype=dtype))
    region = ((1, 3), (16, 48), (0, 96))
    sl = tuple(slice(a, b) for a, b in region)
    x = full[sl].contiguous().to(dev).requires_grad_()
    y = hip.dropout(x, shape, region, key.k0, key.k1, keep)
    y.backward(torch.ones_like(y))
    torch.cuda.synchronize()
    assert torch.equal(y.detach().cpu(), ref[sl])
    gref = torch.where(u[sl] < keep, (torch.ones((), dtype=dtype).float() / keep).to(dtype), torch.zeros((), dtype=dtype))
    assert torch.equal(x.grad.cpu(), gref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_box_slice_backward_is_pad(hip, dtype):
    """box_slice's backward (one pad_box launch) equals torch's slice_backward, for a strided
    incoming gradient too."""
    full = torch.randn(6, 40, 24, dtype=torch.float32).to(dtype).to(dev).requires_grad_()
    box = (slice(2, 5), slice(8, 32), slice(0, 24))
    y = hip.box_slice(full, box)
    assert y.shape == (3, 24, 24)
    g = torch.randn(24, 3, 24, dtype=torch.float32).to(dtype).to(dev).transpose(0, 1)   # non-contiguous
    y.backward(g)
    ref = torch.zeros(6, 40, 24, dtype=dtype, device=dev)
    ref[box] = g
    torch.cuda.synchronize()
    assert torch.equal(full.grad, ref)
    v = torch.randn(640, device=dev).requires_grad_()
    hip.box_slice(v, (slice(320, 640),)).sum().backward()
    assert torch.equal(v.grad, torch.cat([torch.zeros(320, device=dev), torch.ones(320, device=dev)]))


@pytest.mark.parametrize("tile,M,N,K,batch,mode", [
    (2561, 4096, 512, 640, 3, "plain"), (2561, 1000, 384, 512, 1, "bias_relu"), (2562, 4096, 512, 640, 3, "plain"),
    (1602, 4096, 640, 512, 1, "bias_sum"), (1602, 777, 640, 512, 1, "res_add"), (1282, 4096, 512, 640, 1, "mask"),
    (1282, 300, 200, 128, 2, "alpha"), (1284, 2048, 512, 640, 1, "plain"), (12883, 2048, 1536, 640, 1, "plain"),
    (12884, 1024, 256, 192, 1, "res_f32"), (644, 2048, 640, 512, 1, "bias_sum"), (644, 96, 72, 64, 1, "plain")])
def test_gemm_lean_bit_exact(hip, tile, M, N, K, batch, mode):
    """The lean K-loop kernel (gemm.hip gemm_lean_kernel, tile code + 100000) is bit-identical to
    the general LDS-DMA kernel (code + 200000) for every epilogue instance: plain, bias(+ReLU),
    bias + fused sum, alpha, residual add / ReLU mask (bf16 and f32 operand), ragged M / N,
    weight-major batches folded or not, persistent and one-block-per-item grids."""
    A = _rand(M, K, seed=1)
    B = _rand(batch, N, K, seed=2)
    ldc = N * batch if batch > 1 else N
    kw = dict(batch=batch, sA=0, sB=N * K, sC=N) if batch > 1 else {}
    if mode in ("bias_relu", "bias_sum"):
        kw["bias"] = _rand(N, dtype=torch.float32, seed=3)
        kw["relu"] = mode == "bias_relu"
    if mode == "alpha":
        kw["alpha"] = 0.37
    if mode in ("res_add", "mask", "res_f32"):
        kw["res"] = _rand(M, N, dtype=torch.float32 if mode == "res_f32" else torch.bfloat16, seed=4)
        kw["res_ld"] = N
        kw["res_mode"] = "mask" if mode == "mask" else "add"
    outs = {}
    for base in (200000, 100000):
        C = torch.full((M, ldc), float("nan"), device=dev).bfloat16()
        ps = torch.zeros(hip.psum_slots(M, ldc) * 2, device=dev) if mode == "bias_sum" else None
        cnt = hip.gemm(A, B, C, M, N, K, K, K, ldc, True, True, tile=base + tile, psum=ps, **kw)
        torch.cuda.synchronize()
        outs[base] = (C, ps, cnt)
    (c0, p0, n0), (c1, p1, n1) = outs[200000], outs[100000]
    assert torch.equal(c0.view(torch.int16), c1.view(torch.int16))
    assert n0 == n1
    if p0 is not None:
        assert torch.equal(p0[:n0], p1[:n1])
    ref = (A.float() @ B.float().reshape(batch * N, K).t()) if batch > 1 else A.float() @ B[0].float().t()
    if mode == "plain":
        assert ((c1.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2


@pytest.mark.parametrize("B,H,K", [(2, 8, 640), (3, 2, 256), (5, 4, 128)])
def test_qkv_attn_fwd_bit_exact(hip, B, H, K):
    """The fused Q/K/V projection + attention forward (attention.hip qkv_attn_fwd_kernel) writes
    the same Q/K/V bits as the batched projection GEMM (same per-element MFMA sequence) and O / lse
    equal to the resident forward's over those views up to f32 rounding of the softmax state (a
    handful of rows differ by one bf16 ulp: the two kernels' instruction selection for the running
    sum differs), and as close to an fp32 reference; item counts below and above the CU count
    exercise the block's item loop."""
    T, N = B * 256, 64 * H
    x = _rand(T, K, seed=31)
    wt = (_rand(3, N, K, seed=32) * 0.05).contiguous()
    out = torch.full((T, 3 * N), float("nan"), device=dev).bfloat16()
    scale = 64 ** -0.5
    o, lse = hip.qkv_attn_fwd(x, wt, out, H, scale)
    ref = torch.empty_like(out)
    hip.gemm(x, wt, ref, T, N, K, K, K, 3 * N, True, True, batch=3, sA=0, sB=N * K, sC=N)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    q, k, v = (ref.view(B, 256, 3, H, 64)[:, :, i] for i in range(3))
    o_ref, lse_ref = hip.attn_fwd_lse(q, k, v, scale)
    torch.cuda.synchronize()
    o4 = o.view(B, 256, H, 64).float()
    torch.testing.assert_close(o4, o_ref.float(), rtol=0, atol=4e-3)
    assert ((o4 - o_ref.float()).abs().amax(-1) > 0).float().mean().item() < 0.02
    torch.testing.assert_close(lse.view(B, H, 256), lse_ref, rtol=1e-6, atol=1e-5)
    s_ = torch.einsum("bshd,bthd->bhst", q.float(), k.float()) * scale
    o_t = torch.einsum("bhst,bthd->bshd", torch.softmax(s_, -1).bfloat16().float(), v.float())
    assert (o4 - o_t).abs().max().item() <= 1.25 * (o_ref.float() - o_t).abs().max().item() + 1e-3


def test_qkv_attn_fwd_rejects_bad_shapes(hip):
    x = _rand(512, 640)
    wt = _rand(3, 512, 640)
    with pytest.raises(AssertionError):
        hip.qkv_attn_fwd(x[:300], wt, torch.empty(300, 1536, dtype=torch.bfloat16, device=dev), 8, 0.125)
    # the launcher's own checks (K not a multiple of 128)
    rc = hip.lib().ljs_qkv_attn_fwd(hip._p(x), 640, hip._p(wt), hip._p(x), hip._p(x), hip._p(x), 512, 576, 512, 8,
                                    0.125, None, None)
    assert rc != 0


@pytest.mark.parametrize("tile,S", [(1282, 6), (12856, 6), (2563, 4)])
@pytest.mark.parametrize("M,N,T", [(640, 512, 4096), (512, 640, 2048), (320, 200, 640)])
def test_gemm_weight_grad_slab_tiles(hip, tile, S, M, N, T):
    """The weight-gradient (m/n-contiguous operands, f32 split-K slabs) tiles: the slabs sum to the
    fp32 reference C = A^T B over the token dimension, ragged M / N included."""
    A = _rand(T, M, seed=21)
    B = _rand(T, N, seed=22)
    nkt = -(-T // 64)
    Se = hip.slab_count(nkt, S)
    sl = torch.full((Se, M, N), float("nan"), device=dev)
    hip.gemm(A, B, sl, M, N, T, M, N, N, False, False, sC=M * N, splitk=Se, tile=tile, slabs=True)
    torch.cuda.synchronize()
    ref = A.float().t() @ B.float()
    got = sl.sum(0)
    assert not torch.isnan(got).any()
    torch.testing.assert_close(got, ref, rtol=2e-3, atol=2e-3 * ref.abs().max().item())
