"""Sharded checkpoint save / restore (resume on a different mesh)."""
import numpy as np

import learning_jax_sharding_amd as ljs
from learning_jax_sharding_amd import nn, optim
from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh
from learning_jax_sharding_amd.models import MultiHeadAttention
from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P
from learning_jax_sharding_amd.training import TrainState
from learning_jax_sharding_amd.utils import checkpoint as ckpt

RULES = (("batch", "data"), ("embed", "model"), ("hidden", "model"))


def _state(mesh_shape):
    mesh = Mesh(create_device_mesh(mesh_shape), ("data", "model"))
    model = MultiHeadAttention(64, heads=4, dim_head=16)
    x = ljs.random.normal(ljs.random.PRNGKey(0), (4, 32, 64))
    params = model.init(ljs.random.PRNGKey(1), x)["params"]
    params = ljs.device_put(params, nn.logical_to_mesh_sharding(nn.get_partition_spec(params), mesh, RULES))
    st = TrainState.create(apply_fn=model.apply, params=params, tx=optim.adam(1e-2))
    x = ljs.device_put(x, NamedSharding(mesh, P("data", "model")))
    return mesh, model, st, x


def _leaves(st):
    return [np.asarray(l) for l in ljs.tree_util.tree_leaves(nn.unbox(st))]


def test_save_restore_resume_on_other_mesh(host_devices, tmp_path):
    host_devices(4)
    mesh, model, st, x = _state((2, 2))

    def step(st):
        g = ljs.grad(lambda p: model.apply({"params": p}, x).sum())(st.params)
        return st.apply_gradients(grads=g)

    with mesh, nn.axis_rules(RULES):
        st = step(st)
        st = step(st)
    d = ckpt.checkpoint_dir(str(tmp_path), 2)
    ckpt.save_checkpoint(d, st, step=2)
    assert ckpt.latest_step(str(tmp_path)) == 2
    # resume into a differently-sharded target (4 x 1 mesh)
    mesh2, _, target, _ = _state((4, 1))
    restored = ckpt.restore_checkpoint(d, target)
    for a, b in zip(_leaves(restored), _leaves(st)):
        np.testing.assert_array_equal(a, b)
    assert int(np.asarray(restored.step)) == 2
    leaf = ljs.tree_util.tree_leaves(nn.unbox(restored.params))[0]
    assert leaf.sharding.mesh == mesh2


def test_profiler_helpers(host_devices, monkeypatch):
    host_devices(2)
    from learning_jax_sharding_amd import profiler
    mesh = Mesh(create_device_mesh((2,)), ("x",))
    a = ljs.device_put(np.ones((4, 8), np.float32), NamedSharding(mesh, P(None, "x")))
    b = ljs.device_put(np.ones((8, 4), np.float32), NamedSharding(mesh, P("x", None)))
    plan = profiler.collective_plan(lambda a, b: ljs.numpy.matmul(a, b), a, b)
    assert "all_reduce" in plan
    t = profiler.StepTimer().time(lambda: ljs.numpy.matmul(a, b), steps=3, warmup=1).summary()
    assert t["n"] == 3 and t["median_ms"] >= 0
    monkeypatch.setenv("LJS_DEBUG_NANS", "1")
    diff = profiler.compare_sync_async(lambda: ljs.numpy.matmul(a, b), lambda c: [c])
    assert diff == 0.0
    with profiler.annotate("region"):
        pass
    cmd = profiler.rocprof_command(["python3", "bench.py"], "out", counters=["SQ_WAVES"])
    assert cmd[:3] == ["rocprofv3", "--kernel-trace", "--pmc"] and "--" in cmd
