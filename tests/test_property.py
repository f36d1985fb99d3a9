"""Property tests (SURVEY §4 numeric tier): for RANDOM shardings of the operands on random
meshes, every partitioned op equals the unsharded numpy oracle, and the output sharding is
a valid tiling (each device's buffer is exactly its block of the global result)."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

import learning_jax_sharding_amd as ljs
import learning_jax_sharding_amd.numpy as jnp
from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh
from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P, PositionalSharding

MESHES = [((8,), ("x",)), ((2, 4), ("x", "y")), ((4, 2), ("x", "y")), ((2, 2, 2), ("x", "y", "z"))]
SETTINGS = settings(max_examples=20, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])


@st.composite
def spec_for(draw, names, ndim):
    """A PartitionSpec of rank ``ndim`` that uses each mesh axis at most once."""
    free = list(names)
    entries = []
    for _ in range(ndim):
        k = draw(st.integers(0, 2))
        if k == 0 or not free:
            entries.append(None)
            continue
        n = draw(st.integers(1, min(k, len(free))))
        picked = draw(st.permutations(free))[:n]
        for a in picked:
            free.remove(a)
        entries.append(picked[0] if n == 1 else tuple(picked))
    return P(*entries)


def _mesh(shape, names):
    return Mesh(create_device_mesh(shape), names)


def _check_tiling(arr, ref):
    """Each device buffer equals the global oracle at that device's index."""
    assert len(arr.sharding.devices_indices_map(arr.shape)) == len(arr.addressable_shards)
    for shard in arr.addressable_shards:
        np.testing.assert_allclose(np.asarray(shard.data), ref[shard.index], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("mesh_i", range(len(MESHES)))
@SETTINGS
@given(data=st.data())
def test_dot_random_shardings(host_devices, mesh_i, data):
    host_devices(8)
    shape, names = MESHES[mesh_i]
    mesh = _mesh(shape, names)
    sa = data.draw(spec_for(names, 2), "A spec")
    sb = data.draw(spec_for(names, 2), "B spec")
    rng = np.random.default_rng(0)
    A = rng.standard_normal((8, 16)).astype(np.float32)
    B = rng.standard_normal((16, 8)).astype(np.float32)
    a = ljs.device_put(A, NamedSharding(mesh, sa))
    b = ljs.device_put(B, NamedSharding(mesh, sb))
    c = ljs.lax.dot(a, b)
    np.testing.assert_allclose(np.asarray(c), A @ B, rtol=1e-4, atol=1e-4)
    _check_tiling(c, A @ B)


@pytest.mark.parametrize("mesh_i", [1, 3])
@SETTINGS
@given(data=st.data())
def test_einsum_batched_random_shardings(host_devices, mesh_i, data):
    host_devices(8)
    shape, names = MESHES[mesh_i]
    mesh = _mesh(shape, names)
    sa = data.draw(spec_for(names, 3), "A spec")
    sb = data.draw(spec_for(names, 3), "B spec")
    rng = np.random.default_rng(1)
    A = rng.standard_normal((8, 8, 16)).astype(np.float32)
    B = rng.standard_normal((8, 16, 8)).astype(np.float32)
    c = jnp.einsum("ABC,ACD->ABD", ljs.device_put(A, NamedSharding(mesh, sa)),
                   ljs.device_put(B, NamedSharding(mesh, sb)))
    ref = np.einsum("ABC,ACD->ABD", A, B)
    np.testing.assert_allclose(np.asarray(c), ref, rtol=1e-4, atol=1e-4)
    _check_tiling(c, ref)


@pytest.mark.parametrize("mesh_i", [1, 3])
@SETTINGS
@given(data=st.data())
def test_elementwise_reduce_reshard_random(host_devices, mesh_i, data):
    """binary op across differently-sharded operands, reductions, and an explicit reshard."""
    host_devices(8)
    shape, names = MESHES[mesh_i]
    mesh = _mesh(shape, names)
    sa = data.draw(spec_for(names, 3), "A spec")
    sb = data.draw(spec_for(names, 3), "B spec")
    so = data.draw(spec_for(names, 3), "target spec")
    axis = data.draw(st.sampled_from([None, 0, 1, 2, (0, 2)]), "reduce axis")
    rng = np.random.default_rng(2)
    A = rng.standard_normal((8, 8, 8)).astype(np.float32)
    B = rng.standard_normal((8, 8, 8)).astype(np.float32)
    a = ljs.device_put(A, NamedSharding(mesh, sa))
    b = ljs.device_put(B, NamedSharding(mesh, sb))
    s = a * b + a
    np.testing.assert_allclose(np.asarray(s), A * B + A, rtol=1e-5, atol=1e-5)
    r = jnp.sum(s, axis=axis)
    np.testing.assert_allclose(np.asarray(r), np.sum(A * B + A, axis=axis), rtol=1e-4, atol=1e-4)
    t = ljs.with_sharding_constraint(s, NamedSharding(mesh, so))
    assert t.sharding.is_equivalent_to(NamedSharding(mesh, so), 3)
    _check_tiling(t, A * B + A)


@SETTINGS
@given(rep_axis=st.sampled_from([None, 0, 1]), reshape=st.sampled_from([None, (4, 2), (8, 1), (1, 8)]),
       rep2=st.sampled_from([None, 0, 1]))
def test_positional_dot_random(host_devices, rep_axis, reshape, rep2):
    """PositionalSharding layouts not aligned to any mesh axis (case1a's reshape(4,2))."""
    host_devices(8)
    s = PositionalSharding(create_device_mesh((2, 4)))
    sa = s if rep_axis is None else s.replicate(axis=rep_axis, keepdims=True)
    sb = s.reshape(*reshape) if reshape is not None else s
    if rep2 is not None:
        sb = sb.replicate(axis=rep2, keepdims=True)
    rng = np.random.default_rng(3)
    A = rng.standard_normal((8, 16)).astype(np.float32)
    B = rng.standard_normal((16, 8)).astype(np.float32)
    c = ljs.lax.dot(ljs.device_put(A, sa), ljs.device_put(B, sb))
    np.testing.assert_allclose(np.asarray(c), A @ B, rtol=1e-4, atol=1e-4)
    _check_tiling(c, A @ B)
