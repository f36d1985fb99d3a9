"""Every GPU Dense shape runs on a HIP GEMM: f32 compute on the MFMA f32 kernel, unaligned bf16
shapes on the padded MFMA path - no torch GEMM kernel may run."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def no_torch_gemm(monkeypatch):
    def boom(*a, **k):
        raise AssertionError("a torch GEMM ran on the GPU path")
    for name in ("matmul", "mm", "bmm", "addmm", "einsum"):
        monkeypatch.setattr(torch, name, boom)
    monkeypatch.setattr(torch.Tensor, "__matmul__", boom)
    monkeypatch.setattr(torch.Tensor, "matmul", boom)
    yield


@pytest.mark.parametrize("dtype,K,N,bias,relu", [
    (torch.float32, 36, 20, True, False), (torch.float32, 64, 48, False, True),
    (torch.bfloat16, 36, 20, True, True), (torch.bfloat16, 40, 13, False, False)])
def test_dense_unaligned_and_f32_on_hip(gpu_devices, no_torch_gemm, dtype, K, N, bias, relu):
    gpu_devices(1)
    from learning_jax_sharding_amd.ops import hip
    torch.manual_seed(0)
    x = torch.randn(3, 50, K, device="cuda", requires_grad=True)
    w = (torch.randn(K, N, device="cuda") * 0.2).requires_grad_(True)
    b = torch.randn(N, device="cuda", requires_grad=True) if bias else None
    y = hip.linear(x, [w], b, dtype, relu, torch.float32)[0]
    g = torch.randn_like(y)
    (y * g).sum().backward()
    # fp32 oracle of the same op (bf16-rounded operands for bf16 compute)
    xr = x.detach().to(dtype).double().requires_grad_(True)
    wr = w.detach().to(dtype).double().requires_grad_(True)
    br = b.detach().to(dtype).double().requires_grad_(True) if bias else None
    with torch.autograd.set_grad_enabled(True):
        yr = torch.tensordot(xr, wr, dims=1)
        if bias:
            yr = yr + br
        if relu:  # the kernel's own mask: a pre-activation within rounding of 0 may flip
            yr = yr * (y.detach() > 0).double()
        (yr * g.double()).sum().backward()
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=5e-2)
    np.testing.assert_allclose(y.detach().cpu().numpy(), yr.detach().cpu().numpy(), **tol)
    np.testing.assert_allclose(x.grad.cpu().numpy(), xr.grad.cpu().numpy(), **tol)
    np.testing.assert_allclose(w.grad.cpu().numpy(), wr.grad.cpu().numpy(), **tol)
    if bias:
        np.testing.assert_allclose(b.grad.cpu().numpy(), br.grad.cpu().numpy(), **tol)


def test_dense_stack_f32_on_hip(gpu_devices, no_torch_gemm):
    """DenseStack(dtype=float32) - the f32 FSDP test model - trains without torch GEMMs."""
    gpu_devices(1)
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd.models import DenseStack
    model = DenseStack(36, layers=2, dtype=torch.float32)
    x = ljs.random.normal(ljs.random.PRNGKey(0), (2, 8, 36))
    params = model.init(ljs.random.PRNGKey(1), x)["params"]
    val, g = ljs.value_and_grad(lambda p: model.apply({"params": p}, x).sum())(params)
    torch.cuda.synchronize()
    assert np.isfinite(float(np.asarray(val)))
