"""Ping-pong GEMM (csrc/kernels/gemm_pp.hip) vs a plain fp32 torch reference, and bit for bit vs
the LDS-DMA kernels of gemm.hip (same MFMA sequence per 16x16 block: same f32 sums)."""
import math

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


def _rand(*shape, seed=0, dtype=torch.bfloat16):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(*shape, generator=g).to(dtype).to(dev)


# (cfg, M, N, K): whole-tile shapes, ragged M, several items per block (M large), one K-tile
KC_CASES = [(1, 512, 768, 640), (1, 200, 384, 128), (1, 4096, 1536, 640), (2, 384, 640, 512), (2, 136, 320, 64),
            (3, 1024, 512, 640), (3, 264, 256, 192), (4, 512, 512, 256), (5, 512, 512, 640), (5, 300, 256, 128)]


@pytest.mark.parametrize("cfg,M,N,K", KC_CASES)
def test_pp_kc_matches_reference_and_dma_kernel(hip, cfg, M, N, K):
    A = _rand(M, K, seed=1)
    Bt = _rand(N, K, seed=2)                      # [N][K]: k-contiguous B
    ref = A.float() @ Bt.float().t()
    C = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=dev)
    hip.gemm(A, Bt, C, M, N, K, K, K, N, True, True, tile=hip._PP_BASE + cfg)
    C0 = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=dev)
    hip.gemm(A, Bt, C0, M, N, K, K, K, N, True, True, tile=1282)
    torch.cuda.synchronize()
    torch.testing.assert_close(C.float(), ref, rtol=2e-2, atol=2e-2 * math.sqrt(K))
    assert torch.equal(C, C0), (C.float() - C0.float()).abs().max()


def test_pp_bias_relu_alpha_and_fused_sum(hip):
    M, N, K = 520, 640, 512
    A = _rand(M, K, seed=3)
    Bt = _rand(N, K, seed=4)
    for bias_dtype in (torch.float32, torch.bfloat16):
        bias = _rand(N, seed=5, dtype=bias_dtype)
        for relu in (False, True):
            ref = 0.5 * (A.float() @ Bt.float().t()) + bias.float()
            if relu:
                ref = torch.relu(ref)
            C = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=dev)
            ps = torch.zeros(hip.psum_slots(M, N), dtype=torch.float32, device=dev)
            cnt = hip.gemm(A, Bt, C, M, N, K, K, K, N, True, True, bias=bias, relu=relu, alpha=0.5,
                           tile=hip._PP_BASE + 2, psum=ps)
            C0 = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=dev)
            hip.gemm(A, Bt, C0, M, N, K, K, K, N, True, True, bias=bias, relu=relu, alpha=0.5, tile=1282)
            torch.cuda.synchronize()
            torch.testing.assert_close(C.float(), ref, rtol=2e-2, atol=2e-2 * math.sqrt(K))
            assert torch.equal(C, C0)
            assert cnt > 0
            s = ps[:cnt].double().sum().item()
            want = C.double().sum().item()
            assert abs(s - want) <= 1e-3 * max(1.0, abs(want)), (s, want)


def test_pp_qkv_batched_interleaved(hip):
    """The fused QKV call (batch of 3 projections of one activation into interleaved column
    blocks) folds into one [M][3N] GEMM against the stacked weights."""
    M, N, K = 1024, 512, 640
    x = _rand(M, K, seed=6)
    wt = _rand(3, N, K, seed=7)
    out = torch.full((M, 3 * N), float("nan"), dtype=torch.bfloat16, device=dev)
    hip.gemm(x, wt, out, M, N, K, K, K, 3 * N, True, True, batch=3, sA=0, sB=N * K, sC=N, tile=hip._PP_BASE + 1)
    out0 = torch.full((M, 3 * N), float("nan"), dtype=torch.bfloat16, device=dev)
    hip.gemm(x, wt, out0, M, N, K, K, K, 3 * N, True, True, batch=3, sA=0, sB=N * K, sC=N, tile=1282)
    torch.cuda.synchronize()
    assert torch.equal(out, out0)


@pytest.mark.parametrize("cfg", [11, 12, 13])
@pytest.mark.parametrize("S", [1, 3, 8])
def test_pp_weight_grad_slabs(hip, cfg, S):
    """dW = X^T dY with both operands m/n-contiguous, split-K into f32 slabs (uneven last split)."""
    T, Kd, Nd = 2048 + 192, 384, 512
    X = _rand(T, Kd, seed=8)
    dY = _rand(T, Nd, seed=9)
    nkt = T // 64
    S_eff = hip.slab_count(nkt, S)
    slabs = torch.full((S_eff, Kd, Nd), float("nan"), dtype=torch.float32, device=dev)
    hip.gemm(X, dY, slabs, Kd, Nd, T, Kd, Nd, Nd, False, False, sC=Kd * Nd, splitk=S_eff, slabs=True,
             tile=hip._PP_BASE + cfg)
    slabs0 = torch.full((S_eff, Kd, Nd), float("nan"), dtype=torch.float32, device=dev)
    hip.gemm(X, dY, slabs0, Kd, Nd, T, Kd, Nd, Nd, False, False, sC=Kd * Nd, splitk=S_eff, slabs=True, tile=1282)
    torch.cuda.synchronize()
    ref = X.float().t() @ dY.float()
    torch.testing.assert_close(slabs.sum(0), ref, rtol=1e-3, atol=1e-3 * math.sqrt(T))
    assert torch.equal(slabs, slabs0)


def test_pp_weight_grad_bptrs(hip):
    """Slab mode over a batch of separate B tensors (the q / k / v cotangents)."""
    T, Kd, Nd = 1024, 256, 256
    X = _rand(T, Kd, seed=10)
    dys = [_rand(T, Nd, seed=11 + i) for i in range(3)]
    S = 2
    slabs = torch.full((S, 3, Kd, Nd), float("nan"), dtype=torch.float32, device=dev)
    hip.gemm(X, dys[0], slabs, Kd, Nd, T, Kd, Nd, Nd, False, False, batch=3, sA=0, sC=Kd * Nd, splitk=S,
             slabs=True, b_list=dys, tile=hip._PP_BASE + 11)
    torch.cuda.synchronize()
    for i in range(3):
        ref = X.float().t() @ dys[i].float()
        torch.testing.assert_close(slabs[:, i].sum(0), ref, rtol=1e-3, atol=1e-3 * math.sqrt(T))


@pytest.mark.parametrize("M", [1024, 296])
def test_pp_f32_a_cast_fused_and_copy(hip, M):
    """f32 A rounded to bf16 inside the GEMM (cfg 21): bit for bit the GEMM of the cast operand,
    and the bf16 copy written for the backward equals the cast."""
    N, K = 512, 640
    x = _rand(M, K, seed=12, dtype=torch.float32)
    wt = _rand(3, N, K, seed=13)
    out = torch.full((M, 3 * N), float("nan"), dtype=torch.bfloat16, device=dev)
    xb = torch.full((M, K), float("nan"), dtype=torch.bfloat16, device=dev)
    hip.gemm(x, wt, out, M, N, K, K, K, 3 * N, True, True, batch=3, sA=0, sB=N * K, sC=N, acopy=xb,
             tile=hip._PP_BASE + 21)
    ref = torch.full((M, 3 * N), float("nan"), dtype=torch.bfloat16, device=dev)
    hip.gemm(x.bfloat16(), wt, ref, M, N, K, K, K, 3 * N, True, True, batch=3, sA=0, sB=N * K, sC=N, tile=1282)
    torch.cuda.synchronize()
    assert torch.equal(xb, x.bfloat16())
    assert torch.equal(out, ref)


def test_pp_weight_major_batch(hip):
    """A batch of projections into separate [M][N] outputs (the seq-major fused QKV of the 2-D
    layout): one launch over (batch, tiles)."""
    M, N, K = 640, 512, 640
    x = _rand(M, K, seed=14)
    wt = _rand(3, N, K, seed=15)
    out = torch.full((3, M, N), float("nan"), dtype=torch.bfloat16, device=dev)
    hip.gemm(x, wt, out, M, N, K, K, K, N, True, True, batch=3, sA=0, sB=N * K, sC=M * N, tile=hip._PP_BASE + 3)
    out0 = torch.full((3, M, N), float("nan"), dtype=torch.bfloat16, device=dev)
    hip.gemm(x, wt, out0, M, N, K, K, K, N, True, True, batch=3, sA=0, sB=N * K, sC=M * N, tile=1282)
    torch.cuda.synchronize()
    assert torch.equal(out, out0)
