"""Direct peer-memory collectives (comm/p2p.py): kernels vs torch oracles in single-process
``local`` mode (virtual members on the box's GPU) and the multi-process ``ipc`` mode
(scripts/p2p_check.py, ranks sharing the GPU over gloo: IPC buffers, flag barrier, timeout)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("numel,dtype", [(4096, torch.float32), (8 * 1000, torch.bfloat16),
                                         (160 * 1024, torch.float32), (256 * 1024, torch.bfloat16)])
def test_local_group_collectives(dev, n, numel, dtype):
    from learning_jax_sharding_amd.comm.p2p import P2PGroup
    grp = P2PGroup([dev] * n, 1 << 20)
    try:
        xs = {r: torch.randn(numel, device=dev).to(dtype) for r in range(n)}
        ref = xs[0].float()
        for r in range(1, n):
            ref = ref + xs[r].float()
        if grp.fits(numel * xs[0].element_size()):
            out = grp.all_reduce(xs)
            for r in range(n):
                assert torch.equal(out[r], ref.to(dtype)), r
        ag = grp.all_gather(xs)
        for r in range(n):
            assert torch.equal(ag[r], torch.stack([xs[i] for i in range(n)]))
        if numel % (8 * n) == 0:
            c = numel // n
            rs = grp.reduce_scatter({r: x.view(n, c) for r, x in xs.items()})
            a2a = grp.all_to_all({r: x.view(n, c) for r, x in xs.items()})
            for r in range(n):
                assert torch.equal(rs[r], ref.to(dtype).view(n, c)[r])
                assert torch.equal(a2a[r], torch.stack([xs[i].view(n, c)[r] for i in range(n)]))
        grp.check_error()
    finally:
        grp.close()


def test_localcomm_case6_with_p2p_matches_rccl_free_path(gpu_devices, monkeypatch):
    """The case6 attention train step on a 2x2 virtual mesh with LJS_P2P=1 (every collective
    through the peer-memory kernels) == the copy-based loopback path."""
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd.comm.backend import reset_comm
    from learning_jax_sharding_amd import nn
    from learning_jax_sharding_amd.models import MultiHeadAttention
    from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh
    from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P
    import learning_jax_sharding_amd.numpy as jnp

    def run(p2p_on):
        monkeypatch.setenv("LJS_P2P", "1" if p2p_on else "0")
        reset_comm()
        gpu_devices(4)
        mesh = Mesh(create_device_mesh((2, 2)), ("data", "model"))
        rules = (("batch", "data"), ("embed", "model"), ("hidden", "model"))
        model = MultiHeadAttention(128, heads=2, dim_head=64)
        x = ljs.random.normal(ljs.random.PRNGKey(0), (4, 64, 128))
        params = model.init(ljs.random.PRNGKey(1), x)["params"]
        params = ljs.device_put(params, nn.logical_to_mesh_sharding(nn.get_partition_spec(params), mesh, rules))
        x = ljs.device_put(x, NamedSharding(mesh, P("data", "model")))

        def loss(p):
            return model.apply({"params": p}, x).astype(jnp.float32).sum()

        with mesh, nn.axis_rules(rules):
            val, g = ljs.value_and_grad(loss)(params)
        used = bool(getattr(__import__("learning_jax_sharding_amd.comm.backend", fromlist=["get_comm"])
                            .get_comm(), "_p2p_groups", {}))
        return float(np.asarray(val)), [np.asarray(t) for t in ljs.tree_leaves(g)], used

    v0, g0, _ = run(False)
    v1, g1, used = run(True)
    reset_comm()
    assert used, "no collective took the p2p path"
    np.testing.assert_allclose(v1, v0, rtol=1e-3)
    for a, b in zip(g1, g0):
        np.testing.assert_allclose(a.astype(np.float32), b.astype(np.float32), rtol=2e-2, atol=2e-3)


@pytest.mark.parametrize("world", [2, 4])
def test_ipc_group_multiprocess(world):
    env = dict(os.environ, PYTHONPATH=ROOT, LJS_PLATFORM="gpu", LJS_DIST_BACKEND="gloo")
    env.pop("LJS_NUM_DEVICES", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={29631 + world}", os.path.join(ROOT, "scripts", "p2p_check.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    for k in range(world):
        assert f"P2P OK rank {k}" in r.stdout
