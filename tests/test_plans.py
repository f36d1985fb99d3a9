"""Plan tier: the partitioner lowers every case to exactly the collective plan of
SURVEY §2.7 (kinds, device groups, message sizes), on the reference host meshes."""
import numpy as np
import pytest

import learning_jax_sharding_amd as ljs
import learning_jax_sharding_amd.numpy as jnp
from learning_jax_sharding_amd.experimental import mesh_utils
from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh
from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P, PositionalSharding
from learning_jax_sharding_amd.spmd.plan import record_plan

Y_GROUPS = ((0, 1, 2, 3), (4, 5, 6, 7))
X_GROUPS = ((0, 4), (1, 5), (2, 6), (3, 7))


def _groups(step):
    return tuple(tuple(g) for g in step.info["groups"])


def _dot_plan(sa_fn, sb_fn):
    s = PositionalSharding(mesh_utils.create_device_mesh((2, 4)))
    key = ljs.random.PRNGKey(0)
    A = ljs.device_put(ljs.random.normal(key, (4, 16)), sa_fn(s))
    B = ljs.device_put(ljs.random.normal(key, (16, 4)), sb_fn(s))
    with record_plan() as plan:
        C = ljs.lax.dot(A, B)
    np.testing.assert_allclose(np.asarray(C), np.asarray(A) @ np.asarray(B), rtol=1e-5, atol=1e-5)
    return plan, C


def test_plan_case1a(host_devices):
    """1a (case1a.py:24,30): B's contraction blocks follow d//2, A's d%4 -> permute B, then AR
    over Y (the blog's 'mesh axes match' needs a reshard)."""
    host_devices(8)
    plan, C = _dot_plan(lambda s: s.replicate(axis=0, keepdims=True),
                        lambda s: s.reshape(4, 2).replicate(axis=1, keepdims=True))
    st = plan.collectives
    assert [x.kind for x in st] == ["collective_permute", "all_reduce"], plan.as_text()
    # only devices 0 and 7 already hold matching K-blocks: the other 6 receive a block
    assert st[0].info["n_transfers"] == 6
    assert st[1].info["groups"] == Y_GROUPS and st[1].info["bytes_in"] == 64
    assert C.device_buffers[0].shape == (4, 4)


def test_plan_case1b(host_devices):
    """1b (case1b.py:24,30): B's K over X -> slice B to A's K-block locally/exchange, AR over Y."""
    host_devices(8)
    plan, C = _dot_plan(lambda s: s.replicate(axis=0, keepdims=True),
                        lambda s: s.replicate(axis=1, keepdims=True))
    kinds = plan.collective_kinds()
    assert kinds[-1] == "all_reduce" and len(kinds) == 2, plan.as_text()
    assert kinds[0] in ("exchange", "collective_permute")
    assert plan.collectives[-1].info["groups"] == Y_GROUPS and plan.collectives[-1].info["bytes_in"] == 64


def test_plan_case2(host_devices):
    """2 (case2.py:23,29): rows over X, AR over Y of the (2,4) partials (32 B)."""
    host_devices(8)
    plan, C = _dot_plan(lambda s: s, lambda s: s.replicate(axis=1, keepdims=True))
    st = plan.collectives
    assert st[-1].kind == "all_reduce" and st[-1].info["groups"] == Y_GROUPS
    assert st[-1].info["bytes_in"] == 32
    assert C.device_buffers[0].shape == (2, 4)


def test_plan_case3(host_devices):
    """3 (case3_fully_sharded.py:23,29): AG A over Y on K, AG B over X on K, no reduction."""
    host_devices(8)
    plan, C = _dot_plan(lambda s: s, lambda s: s)
    st = plan.collectives
    assert [x.kind for x in st] == ["all_gather", "all_gather"], plan.as_text()
    assert st[0].info["groups"] == Y_GROUPS and st[0].info["dim"] == 1 and st[0].info["bytes_in"] == 32
    assert st[1].info["groups"] == X_GROUPS and st[1].info["dim"] == 0 and st[1].info["bytes_in"] == 32
    assert C.device_buffers[0].shape == (2, 1)


def test_plan_case4(host_devices):
    """4 (case4_gspmd_ff.py:46-52): the GSPMD Fig. 3 FC layer needs NO communication."""
    host_devices(8)
    plan, C = _dot_plan(lambda s: s.replicate(axis=1, keepdims=True),
                        lambda s: s.replicate(axis=0, keepdims=True))
    assert plan.collective_kinds() == [], plan.as_text()
    assert C.addressable_shards[0].data.shape == (2, 1)


def _case5_setup():
    from learning_jax_sharding_amd import nn
    mesh = Mesh(create_device_mesh((2, 2)), ("data", "model"))
    rules = (("batch", "data"), ("embed", "data"), ("hidden", "model"))

    class ToQ(nn.Module):
        inner: int = 32

        @nn.compact
        def __call__(self, x):
            return nn.Dense(self.inner, kernel_init=nn.with_logical_partitioning(
                nn.initializers.lecun_normal(), ("embed", "kv")), use_bias=False, dtype=jnp.bfloat16,
                name="to_q")(x)

    model = ToQ()
    x = ljs.random.normal(ljs.random.PRNGKey(0), (4, 16, 64))
    params = model.init(ljs.random.PRNGKey(1), x)["params"]
    params = ljs.device_put(params, nn.logical_to_mesh_sharding(nn.get_partition_spec(params), mesh, rules))
    x = ljs.device_put(x, NamedSharding(mesh, P("data", "model")))
    return nn, mesh, rules, model, params, x


def test_plan_case5_fsdp(host_devices):
    """5 (case5_attention_dense.py:110): Wq P('data', None) -> forward AG of Wq over data (FSDP);
    backward: the gradient comes back to Wq's sharding through a reduce-scatter over data."""
    host_devices(4)
    nn, mesh, rules, model, params, x = _case5_setup()
    w = params["to_q"]["kernel"]
    assert w.value.device_buffers[0].shape == (32, 32)
    with mesh, nn.axis_rules(rules), record_plan() as fwd:
        model.apply({"params": params}, x)
    st = fwd.collectives
    assert [s.kind for s in st] == ["all_gather"], fwd.as_text()
    assert st[0].info["groups"] == ((0, 2), (1, 3)) and st[0].info["dim"] == 0

    def loss(p):
        return model.apply({"params": p}, x).astype(jnp.float32).sum()

    with mesh, nn.axis_rules(rules), record_plan() as bwd:
        g = ljs.grad(loss)(params)
    kinds = bwd.collective_kinds()
    assert "reduce_scatter" in kinds, bwd.as_text()
    rs = [s for s in bwd.collectives if s.kind == "reduce_scatter"]
    assert any(_groups(s) == ((0, 2), (1, 3)) for s in rs)
    # SURVEY §2.7 "5 bwd": RS over data + AR over model (the replicas of the Wq shard)
    assert any(s.kind == "all_reduce" and _groups(s) == ((0, 1), (2, 3)) for s in bwd.collectives)
    assert g["to_q"]["kernel"].value.sharding.is_equivalent_to(w.value.sharding, 2)


def test_plan_case6_backward(host_devices):
    """6 bwd: the forward's A2A transposes to an A2A; the weight all-gathers
    transpose to reduce-scatters over model; param grads are all-reduced over data."""
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

    def loss(p):
        return model.apply({"params": p}, x).astype(jnp.float32).sum()

    with mesh, nn.axis_rules(rules), record_plan() as plan:
        ljs.grad(loss)(params)
    bwd = [s for s in plan.collectives if s.info.get("note") == "backward"]
    kinds = [s.kind for s in bwd]
    assert "all_to_all" in kinds and "reduce_scatter" in kinds, plan.as_text()
    data_groups = ((0, 2), (1, 3))
    ar = [s for s in plan.collectives if s.kind == "all_reduce"]
    assert ar and all(_groups(s) in (data_groups, ((0, 1, 2, 3),)) for s in ar), plan.as_text()


def test_plan_dp_loss_needs_no_scalar_collectives(host_devices):
    """grad() of a data-parallel loss: the gradient is seeded on the per-shard partial sums,
    so neither the forward all-reduce of the scalar loss nor its transpose runs; the only
    collectives are the gradient replica sums.  value_and_grad() still returns the exact
    all-reduced value (computed when read)."""
    host_devices(4)
    from learning_jax_sharding_amd import nn
    from learning_jax_sharding_amd.models import MultiHeadAttention
    mesh = Mesh(create_device_mesh((4, 1)), ("data", "model"))
    rules = (("batch", "data"), ("embed", "model"), ("hidden", "model"))
    model = MultiHeadAttention(64, heads=4, dim_head=16)
    x = ljs.random.normal(ljs.random.PRNGKey(0), (4, 32, 64))
    params = model.init(ljs.random.PRNGKey(1), x)["params"]
    params = ljs.device_put(params, nn.logical_to_mesh_sharding(nn.get_partition_spec(params), mesh, rules))
    xs = ljs.device_put(x, NamedSharding(mesh, P("data", "model")))

    def loss(p):
        return model.apply({"params": p}, xs).sum()

    with mesh, nn.axis_rules(rules), record_plan() as plan:
        g = ljs.grad(loss)(params)
    notes = [(s.kind, s.info.get("note")) for s in plan.collectives]
    assert all(n == "grad.replica_sum" for _, n in notes), plan.as_text()
    with mesh, nn.axis_rules(rules):
        val, g2 = ljs.value_and_grad(loss)(params)
        ref = float(np.asarray(model.apply({"params": params}, xs).astype(jnp.float32).sum()))
    assert abs(float(np.asarray(val)) - ref) <= 2e-2 * max(1.0, abs(ref))
    for k in ("to_q", "to_out_0"):
        a = np.asarray(nn.unbox(g)[k]["kernel"])
        b = np.asarray(nn.unbox(g2)[k]["kernel"])
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-5)
