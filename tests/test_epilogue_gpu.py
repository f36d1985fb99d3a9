"""GEMM epilogue operand R (residual add / ReLU mask) and its users: bit-exact against the
unfused kernels, and the fused transformer layer / FF block against their unfused forms."""
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


@pytest.mark.parametrize("tile", [64, 128, 2561, 1282, 1284, 12883, 1602])
@pytest.mark.parametrize("M,N,K", [(512, 640, 512), (16384, 640, 640), (304, 136, 128)])
@pytest.mark.parametrize("mode,rdt", [("add", torch.bfloat16), ("add", torch.float32), ("mask", torch.bfloat16)])
def test_gemm_epilogue_operand_bit_exact(hip, tile, M, N, K, mode, rdt):
    A = _rand(M, K, seed=1)
    Bt = _rand(N, K, seed=2)                    # k-contiguous B ([N][K])
    R = _rand(M, N, dtype=rdt, seed=3)
    if mode == "mask":
        R = torch.relu(R)
    bias = _rand(N, dtype=torch.float32, seed=4)
    plain = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
    hip.gemm(A, Bt, plain, M, N, K, K, K, N, True, True, bias=bias, tile=tile)
    fused = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=dev)
    hip.gemm(A, Bt, fused, M, N, K, K, K, N, True, True, bias=bias, tile=tile, res=R, res_ld=N, res_mode=mode)
    torch.cuda.synchronize()
    if mode == "add":
        ref = plain + R.to(torch.bfloat16)          # the unfused bf16 add
    else:
        ref = plain * (R > 0)
    assert torch.equal(fused, ref), (fused.float() - ref.float()).abs().max()


def test_gemm_epilogue_broadcast_row(hip):
    M, N, K = 1024, 640, 512
    A, Bt = _rand(M, K, seed=5), _rand(N, K, seed=6)
    row = _rand(1, N, seed=7)
    plain = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
    hip.gemm(A, Bt, plain, M, N, K, K, K, N, True, True)
    fused = torch.empty_like(plain)
    hip.gemm(A, Bt, fused, M, N, K, K, K, N, True, True, res=row, res_ld=0)
    torch.cuda.synchronize()
    assert torch.equal(fused, plain + row)


def test_linear_residual_autograd(hip):
    x = _rand(4, 128, 512, dtype=torch.float32, seed=8).requires_grad_()
    w = (_rand(512, 640, dtype=torch.float32, seed=9) * 0.05).requires_grad_()
    b = _rand(640, dtype=torch.float32, seed=10).requires_grad_()
    r = _rand(4, 128, 640, dtype=torch.float32, seed=11).requires_grad_()
    (y,) = hip.linear(x, [w], b, torch.bfloat16, False, torch.bfloat16, residual=r)
    g = _rand(4, 128, 640, seed=12)
    (y.float() * g.float()).sum().backward()
    x2, w2, b2, r2 = (t.detach().clone().requires_grad_() for t in (x, w, b, r))
    (y2,) = hip.linear(x2, [w2], b2, torch.bfloat16, False, torch.bfloat16)
    y2 = y2 + r2.to(torch.bfloat16)
    (y2.float() * g.float()).sum().backward()
    assert torch.equal(y, y2)
    for a, c in ((x, x2), (w, w2), (b, b2), (r, r2)):
        torch.testing.assert_close(a.grad, c.grad, rtol=0, atol=0)


def test_ff_block_premasked_relu_backward(hip, monkeypatch):
    """relu(x Win) Wout: the down projection's dX GEMM applies the ReLU mask (fused) and the up
    projection skips its own mask pass; gradients equal the unfused chain's."""
    from learning_jax_sharding_amd.ops import linear as L
    x = _rand(2048, 640, seed=13).requires_grad_()
    w1 = (_rand(640, 2560, dtype=torch.float32, seed=14) * 0.04).requires_grad_()
    w2 = (_rand(2560, 640, dtype=torch.float32, seed=15) * 0.02).requires_grad_()
    g = _rand(2048, 640, seed=16)

    def run(fuse):
        xs, a_, b_ = (t.detach().clone().requires_grad_() for t in (x, w1, w2))
        (h,) = hip.linear(xs, [a_], None, torch.bfloat16, True, torch.bfloat16)
        if not fuse:
            h = h * 1            # a fresh tensor: not registered as a ReLU output
        (y,) = hip.linear(h, [b_], None, torch.bfloat16, False, torch.bfloat16)
        (y.float() * g.float()).sum().backward()
        return y, xs.grad, a_.grad, b_.grad

    calls = []
    for name in ("relu_bwd", "relu_bwd_colsum"):
        orig = getattr(hip, name)
        monkeypatch.setattr(hip, name, lambda *a, _o=orig, _n=name, **k: (calls.append(_n), _o(*a, **k))[1])
    fused = run(True)
    assert calls == [], calls      # no separate mask pass: the dX GEMM applied it
    plain = run(False)
    assert calls == ["relu_bwd"], calls
    for a, c in zip(fused, plain):
        assert torch.equal(a, c), (a.float() - c.float()).abs().max()


@pytest.mark.parametrize("fp8", [False])
def test_transformer_layer_fused_matches_unfused(gpu_devices, monkeypatch, fp8):
    """TransformerLayer (skip connections fused into the out-projection / FF-down epilogues)
    == the same layer written with separate adds."""
    gpu_devices(1)
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd.models import TransformerLayer
    from learning_jax_sharding_amd.ops import core, linear
    # the two forms produce their weight gradients in different orders, so the grouped pairs
    # (ops/linear._hold_dw, jointly chosen split counts) would differ: compared ungrouped
    monkeypatch.setattr(linear, "_DW_GROUP", False)
    model = TransformerLayer(640, heads=8, dim_head=64, ff_dim=2560, fp8=fp8)
    x = ljs.random.normal(ljs.random.PRNGKey(0), (4, 256, 640))
    params = model.init(ljs.random.PRNGKey(1), x)["params"]

    def fused(p):
        return model.apply({"params": p}, x).sum()

    def unfused(p):
        def body(mdl, x):
            h = core.binary("add", core.convert(x, mdl.dtype), mdl.attn(x))
            return core.binary("add", h, mdl.ff(h))
        return model.apply({"params": p}, x, method=body).sum()

    vf, gf = ljs.value_and_grad(fused)(params)
    vu, gu = ljs.value_and_grad(unfused)(params)
    torch.cuda.synchronize()
    # the loss sums the same bf16 values in a different order (fused per-tile partials)
    torch.testing.assert_close(vf.to_torch().float(), vu.to_torch().float(), rtol=1e-4, atol=1e-2)
    lf, lu = ljs.tree_util.tree_leaves(ljs.nn.unbox(gf)), ljs.tree_util.tree_leaves(ljs.nn.unbox(gu))
    for a, b in zip(lf, lu):
        torch.testing.assert_close(a.to_torch(), b.to_torch(), rtol=0, atol=0)



@pytest.mark.parametrize("bcast", [False, True])
@pytest.mark.parametrize("res", [True, False])
def test_ff_block_bf16_matches_unfused(hip, bcast, res):
    """Fused bf16 FF block (one autograd node; skip-path gradient summed in the dX GEMM's
    epilogue) == the unfused dense pair + add, bit for bit."""
    from learning_jax_sharding_amd.ops import linear as L
    T, M, Fd = 2048, 640, 2560
    x = _rand(T, M, seed=70).requires_grad_()
    wi = (_rand(M, Fd, dtype=torch.float32, seed=71) * 0.04).requires_grad_()
    wo = (_rand(Fd, M, dtype=torch.float32, seed=72) * 0.02).requires_grad_()
    cot = torch.ones((), dtype=torch.bfloat16, device=dev).expand(T, M) if bcast else _rand(T, M, seed=73)
    y = L.ff_block(x, wi, wo, res)
    y.backward(cot)
    x2, wi2, wo2 = (t.detach().clone().requires_grad_() for t in (x, wi, wo))
    (h,) = hip.linear(x2, [wi2], None, torch.bfloat16, True, torch.bfloat16)
    (y2,) = hip.linear(h, [wo2], None, torch.bfloat16, False, torch.bfloat16, residual=x2 if res else None)
    y2.backward(cot)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)
    for a, b in ((x.grad, x2.grad), (wi.grad, wi2.grad), (wo.grad, wo2.grad)):
        assert torch.equal(a, b), (a.float() - b.float()).abs().max()


@pytest.mark.parametrize("model_kind", ["attention", "layer", "layer_fp8"])
def test_captured_weight_grads_bit_exact(gpu_devices, model_kind):
    """value_and_grad eagerly == the same gradients from a captured / replayed jit step, bit for bit
    (the deferred weight-gradient combines and grouped dW launches run inside the graph)."""
    gpu_devices(1)
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd.models import MultiHeadAttention, TransformerLayer
    if model_kind == "attention":
        model = MultiHeadAttention(640, 8, 64)
    else:
        model = TransformerLayer(640, heads=8, dim_head=64, ff_dim=2560, fp8=model_kind == "layer_fp8")
    x = ljs.random.normal(ljs.random.PRNGKey(0), (8, 256, 640))
    params = model.init(ljs.random.PRNGKey(1), x)["params"]
    loss = lambda p: model.apply({"params": p}, x).sum()  # noqa: E731
    _, g = ljs.value_and_grad(loss)(params)
    step = ljs.jit(ljs.value_and_grad(loss), capture=True)
    for _ in range(3):
        _, gj = step(params)
    torch.cuda.synchronize()
    eager = [l.to_torch().clone() for l in ljs.tree_util.tree_leaves(ljs.nn.unbox(g))]
    graph = [l.to_torch().clone() for l in ljs.tree_util.tree_leaves(ljs.nn.unbox(gj))]
    for a, b in zip(eager, graph):
        assert torch.equal(a, b), (a.float() - b.float()).abs().max()


@pytest.mark.parametrize("model_kind", ["attention", "layer", "layer_fp8"])
def test_deferred_wgrad_combine_bit_exact(gpu_devices, monkeypatch, model_kind):
    """Weight gradients handed to the fused Adam as their split-K slabs (ops/linear.defer_wgrads:
    no slab_reduce launch) train bit-identically to the combined path, eagerly and under a
    captured/replayed jit step; a gradient read directly is combined on demand (same bits)."""
    gpu_devices(1)
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd import optim
    from learning_jax_sharding_amd.models import MultiHeadAttention, TransformerLayer
    from learning_jax_sharding_amd.ops import linear
    from learning_jax_sharding_amd.training import TrainState
    if model_kind == "attention":
        model = MultiHeadAttention(640, 8, 64)
    else:
        model = TransformerLayer(640, heads=8, dim_head=64, ff_dim=2560, fp8=model_kind == "layer_fp8")
    x = ljs.random.normal(ljs.random.PRNGKey(0), (8, 256, 640))

    def make():
        params = model.init(ljs.random.PRNGKey(1), x)["params"]
        return TrainState.create(apply_fn=model.apply, params=params, tx=optim.adam(1e-3))

    def step(state, x):
        g = ljs.grad(lambda p: model.apply({"params": p}, x).sum())(state.params)
        return state.apply_gradients(grads=g)

    deferred = []
    orig = linear.defer_slabs

    def counting(*a, **k):
        r = orig(*a, **k)
        if r is not None:
            deferred.append(1)
        return r
    monkeypatch.setattr(linear, "defer_slabs", counting)
    orig_ok = linear._defer_ok

    def counting_ok(*a):
        r = orig_ok(*a)
        if r:
            deferred.append(1)
        return r
    monkeypatch.setattr(linear, "_defer_ok", counting_ok)
    # (the grouped weight-gradient pair picks its own split counts, so its sums round differently:
    # compared separately, test_grouped_wgrad_pair_matches_separate)
    monkeypatch.setattr(linear, "_DW_GROUP", False)
    res = {}
    for flag in (False, True):
        monkeypatch.setattr(linear, "_DEFER_ON", flag)
        n0 = len(deferred)
        _, g = ljs.value_and_grad(lambda p: model.apply({"params": p}, x).sum())(make().params)
        se = make()
        for _ in range(2):
            se = step(se, x)
        sj = make()
        jstep = ljs.jit(step, donate_argnums=0, capture=True)
        for _ in range(3):
            sj = jstep(sj, x)
        torch.cuda.synchronize()
        if flag:
            assert len(deferred) > n0, "no weight gradient was deferred"
        else:
            assert len(deferred) == n0
        res[flag] = [l.to_torch().clone() for l in ljs.tree_util.tree_leaves(ljs.nn.unbox(g))] + \
            [np.asarray(l).copy() for l in ljs.tree_util.tree_leaves(se)] + \
            [np.asarray(l).copy() for l in ljs.tree_util.tree_leaves(sj)]
    for a, b in zip(res[False], res[True]):
        if isinstance(a, torch.Tensor):
            assert torch.equal(a, b), (a.float() - b.float()).abs().max()
        else:
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("model_kind", ["attention", "layer"])
def test_grouped_wgrad_pair_matches_separate(gpu_devices, monkeypatch, model_kind):
    """The grouped weight-gradient pair (ops/linear._hold_dw: one grid, jointly chosen split
    counts) trains like the separate launches: same gradients up to the f32 re-association of
    different split counts, under eager and captured steps."""
    gpu_devices(1)
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd import optim
    from learning_jax_sharding_amd.models import MultiHeadAttention, TransformerLayer
    from learning_jax_sharding_amd.ops import hip, linear
    from learning_jax_sharding_amd.training import TrainState
    if model_kind == "attention":
        model = MultiHeadAttention(640, 8, 64)
    else:
        model = TransformerLayer(640, heads=8, dim_head=64, ff_dim=2560)
    x = ljs.random.normal(ljs.random.PRNGKey(0), (8, 256, 640))

    def make():
        params = model.init(ljs.random.PRNGKey(1), x)["params"]
        return TrainState.create(apply_fn=model.apply, params=params, tx=optim.adam(1e-3))

    def step(state, x):
        g = ljs.grad(lambda p: model.apply({"params": p}, x).sum())(state.params)
        return state.apply_gradients(grads=g)

    pairs = []
    orig = hip.pick_dw_pair

    def counting(*a):
        r = orig(*a)
        pairs.append(r)
        return r
    monkeypatch.setattr(hip, "pick_dw_pair", counting)
    res = {}
    for flag in (False, True):
        monkeypatch.setattr(linear, "_DW_GROUP", flag)
        n0 = len(pairs)
        sj = make()
        jstep = ljs.jit(step, donate_argnums=0, capture=True)
        for _ in range(3):
            sj = jstep(sj, x)
        se = step(make(), x)
        torch.cuda.synchronize()
        _, g = ljs.value_and_grad(lambda p: model.apply({"params": p}, x).sum())(make().params)
        torch.cuda.synchronize()
        assert (len(pairs) > n0) == flag and all(p is not None for p in pairs[n0:])
        res[flag] = ([np.asarray(l).copy() for l in ljs.tree_util.tree_leaves(ljs.nn.unbox(g))],
                     [np.asarray(l).copy() for l in ljs.tree_util.tree_leaves(sj)] +
                     [np.asarray(l).copy() for l in ljs.tree_util.tree_leaves(se)])
    # gradients: f32 re-association only
    for a, b in zip(res[False][0], res[True][0]):
        np.testing.assert_allclose(b, a, rtol=1e-4, atol=1e-5 * max(1.0, float(np.abs(a).max())))
    # trained states: Adam normalises each update to ~lr, so a near-zero gradient element whose
    # sign the re-association flips moves by ~lr, and the next steps' gradients are taken at those
    # slightly different weights -- the trajectories agree in norm, not bit for bit
    for a, b in zip(res[False][1], res[True][1]):
        a64, b64 = np.asarray(a, np.float64), np.asarray(b, np.float64)
        assert np.linalg.norm(b64 - a64) <= 5e-2 * max(np.linalg.norm(a64), 1e-12), \
            (np.linalg.norm(b64 - a64), np.linalg.norm(a64))
