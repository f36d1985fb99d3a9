"""Tensor-parallel fused FF block (ops/fp8.ff_block_tp) on host meshes: the reference rules'
('hidden', 'model') split (case6_attention.py:183-187) with x sequence-sharded over 'model'.

The oracle is the single-device fused block on the same weights: the MX-fp8 host emulation
(``_FFBlockFp8Ref``) or the bf16 dense pair.  The TP run differs only in where its partial sums
are rounded (a bf16 partial per hidden slice, summed by the reduce-scatter)."""
import numpy as np
import pytest

import learning_jax_sharding_amd as ljs
from learning_jax_sharding_amd import nn
from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh
from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P

# the FF hidden dim over 'model' (Megatron rules; the reference's own order maps 'embed' first,
# which shards both FF weights along M instead - covered by the gathered-weight test below)
RULES = (("batch", "data"), ("hidden", "model"), ("embed", None))
REF_RULES = (("batch", "data"), ("embed", "model"), ("hidden", "model"))
GSPMD2D = (("batch", "data"), ("embed", "data"), ("heads", "model"), ("hidden", "model"))


def _ff_loss_and_grads(mesh_shape, fp8, B=4, S=64, M=128, F=512, residual=True, rules=RULES):
    from learning_jax_sharding_amd.spmd import plan as _plan
    mesh = Mesh(create_device_mesh(mesh_shape), ("data", "model"))
    model = nn.FeedForward(F, fp8=fp8)
    x = ljs.random.normal(ljs.random.PRNGKey(0), (B, S, M))
    params = model.init(ljs.random.PRNGKey(1), x)["params"]
    params = ljs.device_put(params, nn.logical_to_mesh_sharding(nn.get_partition_spec(params), mesh, rules))
    x = ljs.device_put(x, NamedSharding(mesh, P("data", "model")))

    def loss(p):
        y = model.apply({"params": p}, x, residual=x if residual else None)
        return (y.astype(ljs.numpy.float32) * y.astype(ljs.numpy.float32)).sum()

    with mesh, nn.axis_rules(rules), _plan.record_plan() as rec:
        val, g = ljs.value_and_grad(loss)(params)
    kinds = [st.kind for st in rec.steps]
    return float(np.asarray(val)), ljs.tree_map(lambda a: np.asarray(a), nn.unbox(g)), kinds


@pytest.mark.parametrize("fp8", [True, False])
@pytest.mark.parametrize("mesh_shape", [(2, 2), (1, 4), (1, 2)])
def test_ff_block_tp_matches_single_device(host_devices, fp8, mesh_shape):
    host_devices(4)
    v1, g1, k1 = _ff_loss_and_grads((1, 1), fp8)
    vn, gn, kn = _ff_loss_and_grads(mesh_shape, fp8)
    assert "ff_block" in k1
    assert "ff_block_tp" in kn, kn
    assert abs(v1 - vn) <= 3e-2 * max(1.0, abs(v1)), (v1, vn)
    for name in g1:
        a, b = g1[name], gn[name]
        np.testing.assert_allclose(b, a, rtol=5e-2, atol=5e-2 * np.abs(a).max(), err_msg=name)


@pytest.mark.parametrize("fp8", [True, False])
@pytest.mark.parametrize("rules", ["gspmd2d", "reference"])
def test_ff_block_2d_rules_match_single_device(host_devices, fp8, rules):
    """GSPMD-2D rules (W_in over (data, model): the hidden split TP block with M gathered) and the
    reference rules (both FF weights split along M over 'model': gathered, each device runs the
    fused block on its own tokens)."""
    host_devices(4)
    r = GSPMD2D if rules == "gspmd2d" else REF_RULES
    v1, g1, _ = _ff_loss_and_grads((1, 1), fp8, rules=r, S=128)
    vn, gn, kn = _ff_loss_and_grads((2, 2), fp8, rules=r, S=128)
    assert ("ff_block_tp" if rules == "gspmd2d" else "ff_block") in kn, kn
    assert abs(v1 - vn) <= 3e-2 * max(1.0, abs(v1)), (v1, vn)
    for name in g1:
        a, b = g1[name], gn[name]
        np.testing.assert_allclose(b, a, rtol=5e-2, atol=5e-2 * np.abs(a).max(), err_msg=name)


def test_ff_block_tp_plan_collectives(host_devices):
    """Forward: x gathered over the sequence, W_in resharded to its hidden columns, the partial
    outputs reduce-scattered over 'model'; no all-reduce of activations."""
    host_devices(4)
    _, _, kinds = _ff_loss_and_grads((2, 2), True)
    i = kinds.index("ff_block_tp")
    fwd = kinds[i + 1:i + 3]
    assert fwd == ["all_gather", "reduce_scatter"], kinds
