"""Sharded == unsharded numerics (SURVEY §4 'numeric' tier), on host devices."""
import itertools
import random as pyrandom

import numpy as np
import pytest
import torch

import learning_jax_sharding_amd as ljs
import learning_jax_sharding_amd.numpy as jnp
from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh
from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P
from learning_jax_sharding_amd.spmd.plan import record_plan

AXES = [None, "x", "y", ("x", "y"), ("y", "x")]


def _valid(spec):
    used = [a for p in spec if p is not None for a in ((p,) if isinstance(p, str) else p)]
    return len(used) == len(set(used))


def test_dot_all_layouts(host_devices):
    host_devices(8)
    mesh = Mesh(create_device_mesh((2, 4)), ("x", "y"))
    rng = np.random.default_rng(0)
    A = rng.standard_normal((8, 16)).astype(np.float32)
    B = rng.standard_normal((16, 8)).astype(np.float32)
    ref = A @ B
    combos = [c for c in itertools.product(AXES, repeat=4) if _valid(c[:2]) and _valid(c[2:])]
    pyrandom.Random(0).shuffle(combos)
    for a0, a1, b0, b1 in combos[:60]:
        a = ljs.device_put(A, NamedSharding(mesh, P(a0, a1)))
        b = ljs.device_put(B, NamedSharding(mesh, P(b0, b1)))
        c = ljs.lax.dot(a, b)
        np.testing.assert_allclose(np.asarray(c), ref, rtol=1e-5, atol=1e-4, err_msg=str((a0, a1, b0, b1)))
        # every device holds exactly its tile of the result
        for sh in c.addressable_shards:
            np.testing.assert_allclose(np.asarray(sh.data), ref[sh.index], rtol=1e-5, atol=1e-4)


def test_reshard_roundtrips(host_devices):
    host_devices(8)
    mesh = Mesh(create_device_mesh((2, 4)), ("x", "y"))
    X = np.arange(8 * 8 * 4, dtype=np.float32).reshape(8, 8, 4)
    specs = [P(), P("x"), P("y"), P(None, "y"), P("x", "y"), P("y", "x"), P(("x", "y")), P(None, ("x", "y")),
             P("x", None, "y")]
    for s1, s2 in itertools.product(specs, repeat=2):
        try:
            a = ljs.device_put(X, NamedSharding(mesh, s1))
            b = ljs.device_put(a, NamedSharding(mesh, s2))
        except ValueError:
            continue
        for sh in b.addressable_shards:
            np.testing.assert_array_equal(np.asarray(sh.data), X[sh.index])


def test_reshard_grad_transpose(host_devices):
    """The gradient of a reshard is the transposed collective (AG<->RS, A2A<->A2A, permute)."""
    host_devices(4)
    mesh = Mesh(create_device_mesh((2, 2)), ("x", "y"))
    X = np.random.default_rng(1).standard_normal((4, 8)).astype(np.float32)
    W = np.random.default_rng(2).standard_normal((4, 8)).astype(np.float32)
    for s1, s2 in [(P("x", "y"), P("x")), (P("x"), P(None, "x")), (P(None, "y"), P("y")), (P("y"), P("x"))]:
        a = ljs.device_put(X, NamedSharding(mesh, s1))
        w = ljs.device_put(W, NamedSharding(mesh, s2))

        def f(a):
            b = ljs.with_sharding_constraint(a, NamedSharding(mesh, s2))
            return (b * w).sum()

        g = ljs.grad(f)(a)
        np.testing.assert_allclose(np.asarray(g), W, rtol=1e-6, atol=1e-6, err_msg=str((s1, s2)))


def test_einsum_batched(host_devices):
    host_devices(8)
    rng = np.random.default_rng(0)
    A = rng.standard_normal((8, 4, 16)).astype(np.float32)
    B = rng.standard_normal((8, 16, 4)).astype(np.float32)
    mesh = Mesh(create_device_mesh((2, 4)), ("x", "y"))
    a = ljs.device_put(A, NamedSharding(mesh, P("x", None, "y")))
    b = ljs.device_put(B, NamedSharding(mesh, P("x", "y")))
    c = ljs.numpy.einsum("ABC,ACD->ABD", a, b)
    np.testing.assert_allclose(np.asarray(c), np.einsum("abc,acd->abd", A, B), rtol=1e-5, atol=1e-4)


def _block_loss_and_grads(mesh_shape, impl="fused", fused_qkv=True, B=4, S=32, M=64, heads=4, dh=16):
    from learning_jax_sharding_amd import nn
    from learning_jax_sharding_amd.models import MultiHeadAttention
    n = int(np.prod(mesh_shape))
    mesh = Mesh(create_device_mesh(mesh_shape), ("data", "model"))
    rules = (("batch", "data"), ("embed", "model"), ("hidden", "model"))
    model = MultiHeadAttention(M, heads=heads, dim_head=dh, impl=impl, fused_qkv=fused_qkv)
    x = ljs.random.normal(ljs.random.PRNGKey(0), (B, S, M))
    params = model.init(ljs.random.PRNGKey(1), x)["params"]
    specs = nn.get_partition_spec(params)
    shard = nn.logical_to_mesh_sharding(specs, mesh, rules)
    params = ljs.device_put(params, shard)
    x = ljs.device_put(x, NamedSharding(mesh, P("data", "model")))

    def loss(p):
        return model.apply({"params": p}, x).sum()

    with mesh, nn.axis_rules(rules):
        val, g = ljs.value_and_grad(loss)(params)
    g = nn.unbox(g)
    return float(np.asarray(val)), ljs.tree_map(lambda a: np.asarray(a), g)


@pytest.mark.parametrize("mesh_shape", [(1, 2), (2, 1), (2, 2), (2, 4), (4, 2)])
def test_attention_block_sharded_matches_unsharded(host_devices, mesh_shape):
    host_devices(8)
    v1, g1 = _block_loss_and_grads((1, 1))
    vn, gn = _block_loss_and_grads(mesh_shape)
    assert abs(v1 - vn) <= 2e-2 * max(1.0, abs(v1))
    for k in g1:
        for name in g1[k]:
            a, b = g1[k][name], gn[k][name]
            np.testing.assert_allclose(b, a, rtol=3e-2, atol=3e-2 * np.abs(a).max(), err_msg=f"{k}/{name}")


def test_attention_fused_matches_einsum(host_devices):
    host_devices(4)
    v1, g1 = _block_loss_and_grads((2, 2), impl="einsum", fused_qkv=False)
    v2, g2 = _block_loss_and_grads((2, 2), impl="fused", fused_qkv=True)
    assert abs(v1 - v2) <= 2e-2 * max(1.0, abs(v1))
    for k in g1:
        for name in g1[k]:
            np.testing.assert_allclose(g2[k][name], g1[k][name], rtol=3e-2, atol=3e-2 * np.abs(g1[k][name]).max())


def test_attention_reference_oracle(host_devices):
    """Our fused attention op == a plain torch f32 transcription of case6_attention.py:120-133."""
    host_devices(1)
    from learning_jax_sharding_amd.ops import kernels as K
    g = torch.Generator().manual_seed(0)
    q = torch.randn(2, 16, 4, 8, generator=g).bfloat16()
    k = torch.randn(2, 16, 4, 8, generator=g).bfloat16()
    v = torch.randn(2, 16, 4, 8, generator=g).bfloat16()
    s = torch.einsum("btnh,bfnh->bnft", k.float(), q.float()) * 8 ** -0.5
    p = torch.softmax(s, -1).bfloat16().float()
    ref = torch.einsum("bnft,btnh->bfnh", p, v.float())
    out = K.attention(q, k, v, 8 ** -0.5)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)


def test_adam_matches_torch(host_devices):
    host_devices(2)
    from learning_jax_sharding_amd import optim
    from learning_jax_sharding_amd.training import TrainState
    mesh = Mesh(create_device_mesh((2,)), ("data",))
    rng = np.random.default_rng(0)
    P0 = rng.standard_normal((6, 4)).astype(np.float32)
    G = [rng.standard_normal((6, 4)).astype(np.float32) for _ in range(3)]
    p = {"w": ljs.device_put(P0, NamedSharding(mesh, P("data")))}
    st = TrainState.create(apply_fn=None, params=p, tx=optim.adam(1e-2))
    tp = torch.tensor(P0, requires_grad=True)
    topt = torch.optim.Adam([tp], lr=1e-2, betas=(0.9, 0.999), eps=1e-8)
    for g in G:
        st = st.apply_gradients(grads={"w": ljs.device_put(g, NamedSharding(mesh, P("data")))})
        tp.grad = torch.tensor(g)
        topt.step()
    np.testing.assert_allclose(np.asarray(st.params["w"]), tp.detach().numpy(), rtol=1e-5, atol=1e-6)
    assert int(np.asarray(st.step)) == 3


def test_plan_case6_forward(host_devices):
    """case6 forward lowers to the SURVEY §2.7 plan: AG W, AG K, AG V, AG heads, A2A."""
    host_devices(4)
    from learning_jax_sharding_amd import nn
    from learning_jax_sharding_amd.models import MultiHeadAttention
    mesh = Mesh(create_device_mesh((2, 2)), ("data", "model"))
    rules = (("batch", "data"), ("embed", "model"), ("hidden", "model"))
    model = MultiHeadAttention(64, heads=4, dim_head=16)
    x = ljs.random.normal(ljs.random.PRNGKey(0), (4, 32, 64))
    params = model.init(ljs.random.PRNGKey(1), x)["params"]
    params = ljs.device_put(params, nn.logical_to_mesh_sharding(nn.get_partition_spec(params), mesh, rules))
    x = ljs.device_put(x, NamedSharding(mesh, P("data", "model")))
    with mesh, nn.axis_rules(rules), record_plan() as plan:
        model.apply({"params": params}, x)
    kinds = plan.collective_kinds()
    assert kinds == ["all_gather"] * 6 + ["all_to_all"], kinds


def _layer_loss_and_grads(mesh_shape, fp8, B=4, S=32, M=128, heads=4, dh=32, ff=256):
    from learning_jax_sharding_amd import nn
    from learning_jax_sharding_amd.models import TransformerLayer
    mesh = Mesh(create_device_mesh(mesh_shape), ("data", "model"))
    rules = (("batch", "data"), ("embed", "model"), ("hidden", "model"))
    model = TransformerLayer(M, heads=heads, dim_head=dh, ff_dim=ff, fp8=fp8)
    x = ljs.random.normal(ljs.random.PRNGKey(0), (B, S, M))
    params = model.init(ljs.random.PRNGKey(1), x)["params"]
    params = ljs.device_put(params, nn.logical_to_mesh_sharding(nn.get_partition_spec(params), mesh, rules))
    x = ljs.device_put(x, NamedSharding(mesh, P("data", "model")))

    def loss(p):
        return model.apply({"params": p}, x).astype(jnp.float32).sum()

    with mesh, nn.axis_rules(rules):
        val, g = ljs.value_and_grad(loss)(params)
    return float(np.asarray(val)), ljs.tree_map(lambda a: np.asarray(a), nn.unbox(g))


@pytest.mark.parametrize("fp8", [False, True])
def test_transformer_layer_sharded_matches_unsharded(host_devices, fp8):
    """attention + FF layer (MX-fp8 FF GEMMs when fp8): 2x2 mesh == 1 device.  MX blocks never
    straddle shards (32 | local K), so the fp8 quantization itself is mesh-invariant."""
    host_devices(4)
    v1, g1 = _layer_loss_and_grads((1, 1), fp8)
    v4, g4 = _layer_loss_and_grads((2, 2), fp8)
    assert abs(v1 - v4) <= 2e-2 * max(1.0, abs(v1)), (v1, v4)
    for path in g1:
        for k in g1[path]:
            a, b = g1[path][k], g4[path][k]
            if isinstance(a, dict):
                for n in a:
                    np.testing.assert_allclose(b[n], a[n], rtol=5e-2, atol=5e-2 * np.abs(a[n]).max(),
                                               err_msg=f"{path}/{k}/{n}")
            else:
                np.testing.assert_allclose(b, a, rtol=5e-2, atol=5e-2 * np.abs(a).max(), err_msg=f"{path}/{k}")


def test_fp8_emulation_close_to_bf16(host_devices):
    host_devices(1)
    vb, _ = _layer_loss_and_grads((1, 1), False)
    vf, _ = _layer_loss_and_grads((1, 1), True)
    assert abs(vb - vf) <= 5e-2 * max(1.0, abs(vb)), (vb, vf)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("mesh_shape", [(1, 4), (2, 2)])
def test_ring_attention_matches_allgather(host_devices, causal, mesh_shape):
    """Ring attention (K/V blocks travel, LSE-merged) and Ulysses (sequence <-> heads
    all-to-alls around a local attention) == the all-gather-KV plan, values and gradients, on the
    seq-sharded layout of case6."""
    host_devices(4)
    from learning_jax_sharding_amd.parallel import sequence as SQ
    from learning_jax_sharding_amd.spmd import plan as _plan
    mesh = Mesh(create_device_mesh(mesh_shape), ("data", "model"))
    g = torch.Generator().manual_seed(0)
    B, S, H, D = 2, 32, 4, 16
    arrs = [torch.randn(B, S, H, D, generator=g).bfloat16() for _ in range(3)]
    cot = torch.randn(B, S, H, D, generator=g)
    sh = NamedSharding(mesh, P("data", "model"))
    res = {}
    for mode in ("allgather", "ring", "ulysses"):
        q, k, v = (ljs.device_put(a, sh) for a in arrs)
        leaves = [ljs.spmd.api._fresh_leaf(a) for a in (q, k, v)]
        with _plan.record_plan() as rec:
            out = SQ.context_parallel_attention(*leaves, causal=causal, mode=mode)
        if mode == "ulysses":
            kinds = [st.kind for st in rec.steps]
            assert "ulysses_attention" in kinds and kinds.count("all_to_all") == 4, kinds
        loss = (out.astype(jnp.float32) * ljs.device_put(cot, sh)).sum()
        ins = [t for l in leaves for t in l.local.values()]
        outs = [t for t in loss.local.values()]
        gs = torch.autograd.grad(outs, ins, [torch.full_like(t, 1.0 / len(outs)) for t in outs])
        # assemble per-argument global gradients
        n_loc = len(leaves[0].local)
        glob = []
        for ai, leaf in enumerate(leaves):
            loc = {d: gs[ai * n_loc + i] for i, d in enumerate(leaf.local)}
            from learning_jax_sharding_amd.array import ShardedArray
            ga = ShardedArray(leaf.shape, torch.float32, leaf.sharding, {d: t.float() for d, t in loc.items()})
            glob.append(np.asarray(ga))
        res[mode] = (np.asarray(out.astype(jnp.float32)), glob)
    for mode in ("ring", "ulysses"):
        np.testing.assert_allclose(res[mode][0], res["allgather"][0], rtol=2e-2, atol=2e-2)
        for a, b in zip(res[mode][1], res["allgather"][1]):
            np.testing.assert_allclose(a, b, rtol=3e-2, atol=3e-2 * max(1.0, np.abs(b).max()))


@pytest.mark.parametrize("preset", ["gspmd2d", "megatron", "fsdp"])
def test_rule_presets_match_unsharded(host_devices, preset):
    """The attention block under the GSPMD 2D, Megatron and FSDP rule presets == 1 device."""
    host_devices(4)
    from learning_jax_sharding_amd import nn, parallel
    from learning_jax_sharding_amd.models import MultiHeadAttention

    def run(mesh_shape, rules):
        mesh = Mesh(create_device_mesh(mesh_shape), ("data", "model"))
        model = MultiHeadAttention(64, heads=4, dim_head=16)
        x = ljs.random.normal(ljs.random.PRNGKey(0), (4, 32, 64))
        params = model.init(ljs.random.PRNGKey(1), x)["params"]
        params = ljs.device_put(params, nn.logical_to_mesh_sharding(nn.get_partition_spec(params), mesh, rules))
        x = ljs.device_put(x, NamedSharding(mesh, P("data")))

        def loss(p):
            return model.apply({"params": p}, x).astype(jnp.float32).sum()
        with mesh, nn.axis_rules(rules):
            val, g = ljs.value_and_grad(loss)(params)
        return float(np.asarray(val)), ljs.tree_map(lambda a: np.asarray(a), nn.unbox(g))

    v1, g1 = run((1, 1), parallel.rules(preset))
    v4, g4 = run((2, 2), parallel.rules(preset))
    assert abs(v1 - v4) <= 2e-2 * max(1.0, abs(v1))
    for k in g1:
        for n in g1[k]:
            np.testing.assert_allclose(g4[k][n], g1[k][n], rtol=3e-2, atol=3e-2 * np.abs(g1[k][n]).max())


def test_column_row_parallel_and_fsdp_prefetch(host_devices):
    host_devices(4)
    from learning_jax_sharding_amd.parallel import fsdp, tensor
    mesh = Mesh(create_device_mesh((2, 2)), ("data", "model"))
    rng = np.random.default_rng(0)
    X = rng.standard_normal((8, 16, 32)).astype(np.float32)
    W1 = rng.standard_normal((32, 64)).astype(np.float32) * 0.1
    W2 = rng.standard_normal((64, 32)).astype(np.float32) * 0.1
    ref = np.maximum(X @ W1, 0) @ W2
    with mesh:
        x = ljs.device_put(X, NamedSharding(mesh, P("data")))
        w1 = ljs.device_put(W1, NamedSharding(mesh, P(None, "model")))
        w2 = ljs.device_put(W2, NamedSharding(mesh, P("model", None)))
        h = tensor.column_parallel(x, w1, relu=True, compute_dtype=jnp.float32)
        y = tensor.row_parallel(h, w2, compute_dtype=jnp.float32)
        np.testing.assert_allclose(np.asarray(y), ref, rtol=1e-4, atol=1e-4)
        # FSDP: params sharded over data, gathered on the side (prefetch) before use
        params = fsdp.shard_params({"w1": W1, "w2": W2}, mesh, "data")
        assert params["w1"].tile.tile_shape[1] == 2 or params["w1"].tile.tile_shape[0] == 2
        full = fsdp.Prefetcher(mesh, "data").prefetch(params).wait()
        assert full["w1"].tile.tile_shape == (1, 1)
        y2 = ljs.numpy.matmul(x, full["w1"])
        np.testing.assert_allclose(np.asarray(y2), X @ W1, rtol=1e-4, atol=1e-4)


def test_fp8_ff_block_emulation_matches_reference_recipe(host_devices):
    """The host emulation of the fused MX-fp8 FF block: forward == the two-dense MX-fp8 forward
    (same quantization points), gradients close to an f32 autograd oracle of relu(x Win) Wout
    (fp8 operands everywhere, weight gradients included: loose tolerance), residual gradient
    passed through."""
    host_devices(1)
    from learning_jax_sharding_amd.ops import fp8 as F
    g = torch.Generator().manual_seed(0)
    x = torch.randn(128, 256, generator=g).to(torch.bfloat16).requires_grad_()
    wi = (torch.randn(256, 512, generator=g) * 0.05).requires_grad_()
    wo = (torch.randn(512, 256, generator=g) * 0.05).requires_grad_()
    res = torch.randn(128, 256, generator=g).to(torch.bfloat16).requires_grad_()
    y = F.ff_block_local(x, wi, wo, res)
    a = F.mx_linear_ref(x, wi, None, True, torch.bfloat16)
    y2 = F.mx_linear_ref(a, wo, None, False, torch.bfloat16) + res
    assert torch.equal(y, y2)
    cot = torch.randn(128, 256, generator=g).to(torch.bfloat16)
    (y.float() * cot.float()).sum().backward()
    # vs the straight-through backward of the same fp8 forward (f32 math, the forward's ReLU
    # mask): the fp8 quantization of the backward GEMMs' operands (dY, dA, the weights, and the
    # token-blocked activations of the weight gradients) is the only difference (~5 %)
    a = F.mx_linear_ref(x.detach(), wi.detach(), None, True, torch.bfloat16).float()
    dA = (cot.float() @ wo.detach().t()) * (a > 0)
    want = {"x": dA @ wi.detach().t(), "wi": x.detach().float().t() @ dA, "wo": a.t() @ cot.float()}
    got = {"x": x.grad.float(), "wi": wi.grad, "wo": wo.grad}
    for k, tol in (("x", 0.08), ("wi", 0.08), ("wo", 0.06)):
        err = ((got[k] - want[k]).norm() / want[k].norm()).item()
        assert err < tol, (k, err)
    # and a loose sanity bound against the f32 oracle (mask flips of the fp8 forward included)
    xr, wir, wor = (t.detach().float().requires_grad_() for t in (x, wi, wo))
    (((torch.relu(xr @ wir) @ wor)) * cot.float()).sum().backward()
    for gt, w in ((x.grad.float(), xr.grad), (wi.grad, wir.grad), (wo.grad, wor.grad)):
        assert ((gt - w).norm() / w.norm()).item() < 0.25
    assert torch.equal(res.grad, cot)


@pytest.mark.parametrize("n,spec", [(1, P()), (2, P("x")), (4, P("x", "y"))])
def test_mse_loss_value_and_grad(host_devices, n, spec):
    """ops.core.mse_loss: value and gradient equal torch's mean((y - t)^2) for every sharding
    (the partial sums are all-reduced for the value, seeded directly for the gradient)."""
    host_devices(n)
    from learning_jax_sharding_amd.ops.core import mse_loss
    mesh = Mesh(create_device_mesh((2, 2) if n == 4 else (n, 1)), ("x", "y"))
    rng = np.random.default_rng(3)
    Y = rng.standard_normal((4, 8, 16)).astype(np.float32)
    Tg = rng.standard_normal((4, 8, 16)).astype(np.float32)
    W = rng.standard_normal((16, 16)).astype(np.float32)
    y = ljs.device_put(Y, NamedSharding(mesh, spec))
    t = ljs.device_put(Tg, NamedSharding(mesh, spec))
    w = ljs.device_put(W, NamedSharding(mesh, P()))

    def f(w):
        return mse_loss(ljs.numpy.einsum("bsk,kn->bsn", y, w), t)

    val, g = ljs.value_and_grad(f)(w)
    wt = torch.tensor(W, requires_grad=True)
    ref = ((torch.einsum("bsk,kn->bsn", torch.tensor(Y), wt) - torch.tensor(Tg)) ** 2).mean()
    ref.backward()
    np.testing.assert_allclose(float(np.asarray(val)), float(ref), rtol=1e-5)
    np.testing.assert_allclose(np.asarray(g), wt.grad.numpy(), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("mesh_shape", [(1, 2), (2, 2), (1, 4)])
def test_attention_local_first_kv_gather_matches_unsharded(host_devices, mesh_shape, monkeypatch):
    """Local-first all-gather attention (own K/V block first, remote blocks merged by log-sum-exp,
    backward over the gathered K/V) == the unsharded block, values and gradients."""
    from learning_jax_sharding_amd.ops import core
    host_devices(8)
    v1, g1 = _block_loss_and_grads((1, 1))
    monkeypatch.setattr(core, "_KV_LOCAL_FIRST", "1")
    from learning_jax_sharding_amd.spmd import plan as _plan
    with _plan.record_plan() as rec:
        vn, gn = _block_loss_and_grads(mesh_shape)
    assert any(st.kind == "attention" and st.info.get("local_first") for st in rec.steps), "local-first path not taken"
    assert abs(v1 - vn) <= 2e-2 * max(1.0, abs(v1))
    for k in g1:
        for name in g1[k]:
            a, b = g1[k][name], gn[k][name]
            np.testing.assert_allclose(b, a, rtol=3e-2, atol=3e-2 * np.abs(a).max(), err_msg=f"{k}/{name}")


def test_loss_seed_hoisted_through_output_all_to_all(host_devices, monkeypatch):
    """The reference's final ('batch', 'embed') constraint is an all-to-all; grad() of the block's
    sum seeds the all-to-all's inputs instead (the sum is permutation-invariant): same value and
    gradients as seeding the outputs."""
    from learning_jax_sharding_amd.spmd import api
    host_devices(4)
    n0 = api.HOIST_STATS["hoisted"]
    v1, g1 = _block_loss_and_grads((2, 2))
    assert api.HOIST_STATS["hoisted"] > n0
    monkeypatch.setattr(api, "_SEED_HOIST", False)
    v0, g0 = _block_loss_and_grads((2, 2))
    assert abs(v1 - v0) <= 1e-3 * max(1.0, abs(v0))
    for k in g0:
        for name in g0[k]:
            np.testing.assert_allclose(g1[k][name], g0[k][name], rtol=1e-4, atol=1e-5, err_msg=f"{k}/{name}")


def test_all_to_all_node_keeps_no_activation(host_devices):
    """The all-to-all's autograd node keeps only its inputs' metadata for the seed hoist (the
    activations themselves are not held until the backward)."""
    import torch
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd.comm import collectives as C
    host_devices(2)
    xs = {d: torch.randn(4, 6, requires_grad=True) * 1.0 for d in (0, 1)}
    spec = C._Spec("all_to_all", [(0, 1)], split_dim=0, concat_dim=1)
    outs = C._CollectiveFn.apply(spec, (0, 1), (0, 1), xs[0], xs[1])
    meta = outs[0].grad_fn.perm_inputs
    assert meta is not None and not any(isinstance(v, torch.Tensor) for m in meta for v in m)
    assert meta[0][0] == (4, 6)


def test_loss_seed_hoist_onto_leaf_inputs(host_devices, monkeypatch):
    """The seed hoist when the all-to-all's inputs are themselves the differentiated leaves (their
    edges are AccumulateGrad nodes): grad of sum(reshard(p)) is all ones, hoisted or not."""
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh
    from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P
    from learning_jax_sharding_amd.spmd import api
    host_devices(4)
    mesh = Mesh(create_device_mesh((4, 1)), ("data", "model"))
    p = ljs.device_put(ljs.random.normal(ljs.random.PRNGKey(0), (16, 32)), NamedSharding(mesh, P("data", None)))

    def loss(x):
        return ljs.lax.with_sharding_constraint(x, NamedSharding(mesh, P(None, "data"))).sum()

    res = {}
    for hoist in (True, False):
        monkeypatch.setattr(api, "_SEED_HOIST", hoist)
        n0 = api.HOIST_STATS["hoisted"]
        val, g = ljs.value_and_grad(loss)(p)
        res[hoist] = (float(np.asarray(val)), np.asarray(g), api.HOIST_STATS["hoisted"] - n0)
    assert res[True][2] > 0 and res[False][2] == 0
    np.testing.assert_allclose(res[True][0], float(np.asarray(p).sum()), rtol=1e-5)
    np.testing.assert_array_equal(res[True][1], np.ones((16, 32), np.float32))
    np.testing.assert_array_equal(res[False][1], res[True][1])
