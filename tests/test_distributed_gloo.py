"""Multi-process SPMD (one device per process) over gloo: the exact code path the
8-GPU RCCL run takes (DistComm, process groups per device group, P2P exchange)."""
import os
import pickle
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _worker(rank, world, port, out_dir, job):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "LJS_PLATFORM": "cpu"})
    os.environ.pop("LJS_NUM_DEVICES", None)
    torch.set_num_threads(1)
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd.runtime.devices import reset_backend
    reset_backend()
    ljs.initialize_distributed()
    reset_backend()
    res = globals()[job](ljs)
    with open(os.path.join(out_dir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(res, f)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def job_collectives(ljs):
    from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh
    from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P
    assert ljs.device_count() == 2 and ljs.local_device_count() == 1
    mesh = Mesh(create_device_mesh((2,)), ("x",))
    X = np.arange(4 * 6, dtype=np.float32).reshape(4, 6)
    out = {}
    for s1, s2 in [(P("x"), P()), (P("x"), P(None, "x")), (P(), P("x")), (P(None, "x"), P("x"))]:
        a = ljs.device_put(X, NamedSharding(mesh, s1))
        b = ljs.device_put(a, NamedSharding(mesh, s2))
        out[str((s1, s2))] = np.asarray(b)
    A = np.random.default_rng(0).standard_normal((4, 8)).astype(np.float32)
    B = np.random.default_rng(1).standard_normal((8, 6)).astype(np.float32)
    a = ljs.device_put(A, NamedSharding(mesh, P(None, "x")))
    b = ljs.device_put(B, NamedSharding(mesh, P("x", None)))
    out["dot"] = np.asarray(ljs.lax.dot(a, b))
    out["dot_ref"] = A @ B
    return out


def job_train(ljs, shapes=((2, 1), (1, 2)), batch=4, seq=32, dtype=torch.bfloat16, rules=None):
    from learning_jax_sharding_amd import nn, optim
    from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh
    from learning_jax_sharding_amd.models import MultiHeadAttention
    from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P
    from learning_jax_sharding_amd.training import TrainState
    res = {}
    for shape in shapes:
        mesh = Mesh(create_device_mesh(shape), ("data", "model"))
        if rules is None:
            rules = (("batch", "data"), ("embed", "model"), ("hidden", "model"))
        model = MultiHeadAttention(64, heads=4, dim_head=16, dtype=dtype)
        x = ljs.random.normal(ljs.random.PRNGKey(0), (batch, seq, 64))
        params = model.init(ljs.random.PRNGKey(1), x)["params"]
        params = ljs.device_put(params, nn.logical_to_mesh_sharding(nn.get_partition_spec(params), mesh, rules))
        x = ljs.device_put(x, NamedSharding(mesh, P("data", "model")))
        state = TrainState.create(apply_fn=model.apply, params=params, tx=optim.adam(1e-3))

        def step(state, x):
            def loss(p):
                return model.apply({"params": p}, x).sum()
            l, g = ljs.value_and_grad(loss)(state.params)
            return state.apply_gradients(grads=g), l

        with mesh, nn.axis_rules(rules):
            for _ in range(2):
                state, l = step(state, x)
        res[str(shape)] = (float(np.asarray(l)),
                           {k: np.asarray(v["kernel"].value if hasattr(v["kernel"], "value") else v["kernel"])
                            for k, v in state.params.items()})
    return res


# the reference's meshes: 2x2 (case5/6, 4 devices) and 2x4 (cases 1-4, 8 devices), plus the
# transposed / 1-D layouts, so every mesh axis has several groups and cross-process
# all-to-all, exchange (batch_isend_irecv) and per-axis sub-groups all run
MESHES = {4: ((2, 2), (1, 4), (4, 1)), 8: ((2, 4), (4, 2), (1, 8))}


def _job_meshes(ljs, world):
    return {"f32": job_train(ljs, MESHES[world], batch=8, seq=32, dtype=torch.float32),
            "bf16": job_train(ljs, MESHES[world], batch=8, seq=32)}


def job_train_w4(ljs):
    return _job_meshes(ljs, 4)


def job_train_w8(ljs):
    return _job_meshes(ljs, 8)


def job_train_overlap_fp32(ljs):
    os.environ.update({"LJS_OVERLAP_GRAD_REDUCE": "force", "LJS_GRAD_COMM_DTYPE": "fp32"})
    return _overlap_train(ljs)


def job_train_overlap_bf16(ljs):
    os.environ.update({"LJS_OVERLAP_GRAD_REDUCE": "force", "LJS_GRAD_COMM_DTYPE": "bf16"})
    return _overlap_train(ljs)


def _overlap_train(ljs):
    """The overlapped bucketed reducer (parallel/data.py) on host tensors: producer groups,
    buckets and the wire dtype, with the collectives recorded in the plan."""
    from learning_jax_sharding_amd.spmd import plan as _plan
    with _plan.record_plan() as rec:
        res = job_train(ljs)
    res["buckets"] = [(s.info.get("dtype"), s.info.get("bytes_in")) for s in rec.steps
                      if s.info.get("note") == "grad.bucket"]
    return res


def _run(job, world=2):
    port = 29500 + (os.getpid() % 1000) + 7 * world
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, port, d, job), nprocs=world, join=True)
        out = []
        for r in range(world):
            with open(os.path.join(d, f"r{r}.pkl"), "rb") as f:
                out.append(pickle.load(f))
    return out


def test_dist_collectives():
    r0, r1 = _run("job_collectives")
    X = np.arange(24, dtype=np.float32).reshape(4, 6)
    for k in r0:
        if k.startswith("dot"):
            continue
        np.testing.assert_array_equal(r0[k], X)
        np.testing.assert_array_equal(r1[k], X)
    np.testing.assert_allclose(r0["dot"], r0["dot_ref"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(r1["dot"], r0["dot_ref"], rtol=1e-5, atol=1e-5)


def test_dist_train_matches_single_process(host_devices):
    r0, r1 = _run("job_train")
    # single-process reference on 2 host devices
    host_devices(2)
    import learning_jax_sharding_amd as ljs
    ref = job_train(ljs)
    for shape in ref:
        lref, pref = ref[shape]
        for r in (r0, r1):
            l, p = r[shape]
            assert abs(l - lref) <= 1e-2 * max(1, abs(lref)), (shape, l, lref)
            for k in pref:
                np.testing.assert_allclose(p[k], pref[k], rtol=1e-4, atol=1e-5)


def _adam_close(a, b, what):
    """Parameters after 2 Adam steps from gradients that differ only by rounding: an element
    whose gradient is ~0 may take the opposite step (|update| <= lr = 1e-3 per step)."""
    diff = np.abs(a - b)
    assert diff.max() <= 4.2e-3, (what, diff.max())
    assert np.mean(diff > 2e-3 + 2e-2 * np.abs(b)) < 1e-2, what


@pytest.mark.parametrize("world", [4, 8])
def test_dist_train_reference_meshes(host_devices, world):
    """case6 train steps on the reference's 2x2 / 2x4 meshes (and their transposes / 1-D
    layouts) with one gloo process per device:
    * f32 compute == the same SPMD job on in-process host devices to f32 tolerance (same
      partition, same math; only the collectives' summation order differs);
    * bf16 compute (the reference dtype) == the in-process job and an unsharded 1x1 run up to
      bf16 partial-sum rounding (gloo sums bf16 collectives in bf16, the loopback in f32)."""
    outs = _run(f"job_train_w{world}", world=world)
    host_devices(world)
    import learning_jax_sharding_amd as ljs
    ref32 = job_train(ljs, MESHES[world], batch=8, seq=32, dtype=torch.float32)
    ref16 = job_train(ljs, MESHES[world], batch=8, seq=32)
    host_devices(1)
    one = job_train(ljs, ((1, 1),), batch=8, seq=32)["(1, 1)"]
    for shape in ref32:
        lref, pref = ref32[shape]
        for r in outs:
            l, p = r["f32"][shape]
            assert abs(l - lref) <= 1e-4 * max(1, abs(lref)), (shape, l, lref)
            for k in pref:
                np.testing.assert_allclose(p[k], pref[k], rtol=1e-4, atol=1e-5, err_msg=f"{shape} {k}")
        lref, pref = ref16[shape]
        l1, p1 = one
        for r in outs:
            l, p = r["bf16"][shape]
            assert abs(l - lref) <= 1e-2 * max(1, abs(lref)), (shape, l, lref)
            for k in pref:
                _adam_close(p[k], pref[k], (shape, k))
        assert abs(lref - l1) <= 3e-2 * max(1, abs(l1)), (shape, lref, l1)
        for k in p1:
            _adam_close(pref[k], p1[k], (shape, k, "1x1"))


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_dist_train_overlapped_reducer(host_devices, wire):
    r0, r1 = _run(f"job_train_overlap_{wire}")
    host_devices(2)
    import learning_jax_sharding_amd as ljs
    ref = job_train(ljs)
    # (2,1): DP over 2 ranks -> bucketed grad all-reduce; the out-projection bucket and the
    # Q/K/V producer group (one [3,K,N] buffer, reduced in place) per step
    assert r0["buckets"] and all(dt == ("bfloat16" if wire == "bf16" else "float32") for dt, _ in r0["buckets"])
    tol = dict(rtol=1e-4, atol=1e-5) if wire == "fp32" else dict(rtol=2e-2, atol=2e-4)
    for shape in ref:
        lref, pref = ref[shape]
        for r in (r0, r1):
            l, p = r[shape]
            assert abs(l - lref) <= 1e-2 * max(1, abs(lref)), (shape, l, lref)
            for k in pref:
                np.testing.assert_allclose(p[k], pref[k], **tol)


def job_train_fsdp(ljs, mesh_shape=(2, 1)):
    """case3 at scale (bench.py --model fsdp): every weight and Adam moment sharded over
    'data'; DenseStack prefetches each layer's gather (parallel.fsdp.Prefetcher) and autograd
    reduce-scatters the gradients."""
    from learning_jax_sharding_amd import nn, optim
    from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh
    from learning_jax_sharding_amd.models import DenseStack
    from learning_jax_sharding_amd.parallel import fsdp
    from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P
    from learning_jax_sharding_amd.spmd import plan as _plan
    from learning_jax_sharding_amd.training import TrainState
    mesh = Mesh(create_device_mesh(mesh_shape), ("data", "model"))
    model = DenseStack(64, layers=3, dtype=torch.float32)
    x = ljs.random.normal(ljs.random.PRNGKey(0), (4, 16, 64))

    def init_fn(k, x):
        return TrainState.create(apply_fn=model.apply, params=model.init(k, x)["params"], tx=optim.adam(1e-3))

    abstract = ljs.eval_shape(init_fn, ljs.random.PRNGKey(1), x)
    shard = fsdp.fsdp_shardings(abstract, mesh, "data")
    state = ljs.jit(init_fn, out_shardings=shard)(ljs.random.PRNGKey(1), x)
    x = ljs.device_put(x, NamedSharding(mesh, P("data")))

    def step(state, x):
        def loss(p):
            return model.apply({"params": p}, x).sum()
        l, g = ljs.value_and_grad(loss)(state.params)
        return state.apply_gradients(grads=g), l

    with mesh, _plan.record_plan() as rec:
        for _ in range(2):
            state, l = step(state, x)
    ker = {k: v["kernel"] for k, v in state.params.items()}
    notes = [st.info.get("note") for st in rec.steps]
    return (float(np.asarray(l)), {k: np.asarray(v) for k, v in ker.items()},
            {k: tuple(v.tile.tile_shape) for k, v in ker.items()}, rec.collective_kinds() + notes)


def test_dist_train_fsdp(host_devices):
    r0, r1 = _run("job_train_fsdp")
    host_devices(2)
    import learning_jax_sharding_amd as ljs
    lref, pref, tiles, kinds = job_train_fsdp(ljs)
    assert any("gather" in str(k) for k in kinds) and any("reduce_scatter" in str(k) for k in kinds), kinds
    assert "fsdp.prefetch" in kinds, kinds  # the gathers come from the prefetcher
    # and the sharded job equals unsharded training on one device (f32 compute)
    host_devices(1)
    l1, p1, _, kinds1 = job_train_fsdp(ljs, (1, 1))
    assert "fsdp.prefetch" not in kinds1
    for l, p, t, k_r in (r0, r1):
        assert "fsdp.prefetch" in k_r
        assert abs(l - lref) <= 1e-3 * max(1, abs(lref)), (l, lref)
        assert abs(l - l1) <= 1e-3 * max(1, abs(l1)), (l, l1)
        assert all(2 in ts for ts in t.values()), t  # weights stay sharded over 'data'
        for k in pref:
            np.testing.assert_allclose(p[k], pref[k], rtol=1e-4, atol=1e-5)
            np.testing.assert_allclose(p[k], p1[k], rtol=1e-4, atol=1e-5)


def job_train_case5(ljs):
    """The attention block under the case5 rules (embed -> data, case5_attention_dense.py:109-112):
    Wq/Wk/Wv/Wo sharded FSDP-style over 'data' and gathered at use (bench.py --rules case5)."""
    from learning_jax_sharding_amd.parallel.tensor import FSDP_RULES
    return job_train(ljs, ((2, 1), (1, 2)), batch=4, seq=32, dtype=torch.float32, rules=FSDP_RULES)


def test_dist_train_case5_rules_matches_unsharded(host_devices):
    r0, r1 = _run("job_train_case5")
    host_devices(1)
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd.parallel.tensor import FSDP_RULES
    l1, p1 = job_train(ljs, ((1, 1),), batch=4, seq=32, dtype=torch.float32, rules=FSDP_RULES)["(1, 1)"]
    for r in (r0, r1):
        for shape, (l, p) in r.items():
            assert abs(l - l1) <= 1e-4 * max(1, abs(l1)), (shape, l, l1)
            for k in p1:
                np.testing.assert_allclose(p[k], p1[k], rtol=1e-4, atol=1e-5, err_msg=f"{shape} {k}")
