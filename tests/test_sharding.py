"""Unit tests of the sharding algebra (SURVEY §4 'unit' tier)."""
import numpy as np
import pytest

from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P, PositionalSharding, TileAssignment
from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh
from learning_jax_sharding_amd.nn import partitioning as nnp


def test_positional_replicate_and_reshape(host_devices):
    host_devices(8)
    s = PositionalSharding(create_device_mesh((2, 4)))
    a = s.replicate(axis=0, keepdims=True)
    assert a.shape == (1, 4)
    ta = a.tile_assignment(2)
    assert ta.tile_shape == (1, 4) and ta.num_replicas == 2
    assert [ta.holders((0, j)) for j in range(4)] == [(0, 4), (1, 5), (2, 6), (3, 7)]
    b = s.reshape(4, 2).replicate(axis=1, keepdims=True)
    tb = b.tile_assignment(2)
    assert [tb.holders((i, 0)) for i in range(4)] == [(0, 1), (2, 3), (4, 5), (6, 7)]
    # case1a hazard: contraction blocks agree only on devices 0 and 7
    agree = [d for d in range(8) if ta.coords[d][1] == tb.coords[d][0]]
    assert agree == [0, 7]


def test_shard_shapes_cases(host_devices):
    host_devices(8)
    s = PositionalSharding(create_device_mesh((2, 4)))
    assert s.replicate(0).shard_shape((4, 16)) == (4, 4)
    assert s.reshape(4, 2).replicate(1).shard_shape((16, 4)) == (4, 4)
    assert s.replicate(1).shard_shape((16, 4)) == (8, 4)
    assert s.shard_shape((4, 16)) == (2, 4)
    assert s.shard_shape((16, 4)) == (8, 1)


def test_named_sharding_tile(host_devices):
    devs = host_devices(4)
    mesh = Mesh(create_device_mesh((2, 2)), ("data", "model"))
    x = NamedSharding(mesh, P("data", "model"))
    ta = x.tile_assignment(3)
    assert ta.tile_shape == (2, 2, 1) and ta.num_replicas == 1
    assert x.shard_shape((8, 256, 640)) == (4, 128, 640)
    w = NamedSharding(mesh, P("model", None))
    tw = w.tile_assignment(2)
    assert tw.tile_shape == (2, 1) and tw.holders((0, 0)) == (0, 2)
    rep = NamedSharding(mesh, P(None))
    assert rep.tile_assignment(2).is_fully_replicated
    with pytest.raises(ValueError):
        NamedSharding(mesh, P("data", "data"))


def test_devices_indices_map(host_devices):
    host_devices(4)
    mesh = Mesh(create_device_mesh((2, 2)), ("x", "y"))
    m = NamedSharding(mesh, P("x")).devices_indices_map((4, 6))
    idx = {d.id: v for d, v in m.items()}
    assert idx[0] == (slice(0, 2), slice(0, 6)) and idx[3] == (slice(2, 4), slice(0, 6))


def test_groups_along(host_devices):
    host_devices(4)
    mesh = Mesh(create_device_mesh((2, 2)), ("data", "model"))
    ta = NamedSharding(mesh, P("data", "model")).tile_assignment(2)
    assert ta.groups_along([1]) == [(0, 1), (2, 3)]
    assert ta.groups_along([0]) == [(0, 2), (1, 3)]
    assert ta.groups_along([0, 1]) == [(0, 1, 2, 3)]


def test_logical_rules():
    rules = (("batch", "data"), ("embed", "model"), ("hidden", "model"))
    assert tuple(nnp.logical_to_mesh_axes(("embed", "heads"), rules)) == ("model", None)
    assert tuple(nnp.logical_to_mesh_axes(("heads", "embed"), rules)) == (None, "model")
    assert tuple(nnp.logical_to_mesh_axes(("batch", "embed", None), rules)) == ("data", "model", None)
    # a mesh axis is used at most once per array
    assert tuple(nnp.logical_to_mesh_axes(("embed", "hidden"), rules)) == ("model", None)
    rules5 = (("batch", "data"), ("embed", "data"), ("hidden", "model"))
    assert tuple(nnp.logical_to_mesh_axes(("embed", "kv"), rules5)) == ("data", None)
    assert tuple(nnp.logical_to_mesh_axes(("batch", "embed"), rules5)) == ("data", None)


def test_tile_assignment_from_coords():
    ta = TileAssignment.from_coords({0: (0,), 1: (1,), 2: (0,), 3: (1,)}, (2,))
    assert ta.holders((0,)) == (0, 2)
    assert TileAssignment.from_coords({0: (0,), 1: (0,), 2: (0,), 3: (1,)}, (2,)) is None


def test_hybrid_device_mesh(host_devices, monkeypatch):
    """mesh_utils.create_hybrid_device_mesh: the dcn factor of each axis spans nodes (outer), the
    per-node factor a node's devices; nodes from LOCAL_WORLD_SIZE process groups, or consecutive
    blocks of one process's devices."""
    from learning_jax_sharding_amd.experimental import mesh_utils
    from learning_jax_sharding_amd import mesh as M
    host_devices(8)
    m = mesh_utils.create_hybrid_device_mesh((1, 4), (2, 1))
    assert [[d.id for d in r] for r in m] == [[0, 1, 2, 3], [4, 5, 6, 7]]
    m = mesh_utils.create_hybrid_device_mesh((2, 2), (1, 2))
    assert [[d.id for d in r] for r in m] == [[0, 1, 4, 5], [2, 3, 6, 7]]
    with pytest.raises(ValueError):
        mesh_utils.create_hybrid_device_mesh((2, 4), (2, 1))
    # nodes from process groups: 4 processes x 2 devices, 2 processes per node
    class D:
        def __init__(self, i):
            self.id, self.process_index = i, i // 2
    devs = [D(i) for i in range(8)]
    monkeypatch.setenv("LJS_LOCAL_WORLD_SIZE", "2")
    m = M.create_hybrid_device_mesh((2, 2), (2, 1), devices=devs)
    assert [[d.id for d in r] for r in m] == [[0, 1], [2, 3], [4, 5], [6, 7]]
    assert [M.node_of(d) for d in devs] == [0, 0, 0, 0, 1, 1, 1, 1]


def test_debug_print_and_callback(host_devices, capsys):
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd import debug
    host_devices(4)
    mesh = Mesh(create_device_mesh((2, 2)), ("a", "b"))
    x = ljs.device_put(ljs.numpy.arange(8.0).reshape(2, 4), NamedSharding(mesh, P("a", "b")))
    debug.print("sum={s} first={}", x[0, 0], s=x.sum())
    seen = []
    debug.callback(lambda v, k=None: seen.append((v.shape, float(k))), x, k=x.sum())
    assert capsys.readouterr().out.strip() == "sum=28.0 first=0.0"
    assert seen == [((2, 4), 28.0)]
    assert ljs.numpy.arange(8).dtype == ljs.numpy.int32 and ljs.numpy.arange(0, 2, 0.5).shape == (4,)
