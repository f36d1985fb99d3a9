"""Single-controller capture (spmd/graphs.py MultiDeviceGraph) through the REAL torch / HIP
backend (``_TorchMD``) on one MI355X: a 2-way data-parallel train step over two virtual devices
of GPU 0 (its gradient all-reduce is a LocalComm collective issued inside the capture) is
captured as a MultiDeviceGraph([0]), replayed, and must match the eager steps (same tolerance as test_gpu_e2e's one-device capture).

This is the one-device case of the reference's execution model (one process driving every
device, ``case6_attention.py:4-5,219-220``); the cross-device fork is covered by the recording
mock in tests/test_multi_gpu_capture.py."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_multi_device_graph_real_backend_matches_eager(gpu_devices, monkeypatch):
    gpu_devices(2)
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd import nn, optim
    from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh
    from learning_jax_sharding_amd.models import MultiHeadAttention
    from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P
    from learning_jax_sharding_amd.spmd import api, graphs
    from learning_jax_sharding_amd.training import TrainState

    made = []
    real = graphs.MultiDeviceGraph

    class _Probe(real):
        def __init__(self, devs, backend=None):
            super().__init__(devs, backend)
            made.append(self)

    monkeypatch.setattr(api, "_MULTI_GPU_CAPTURE", True)
    monkeypatch.setattr(api, "_spans_gpus", lambda: True)
    monkeypatch.setattr(graphs, "MultiDeviceGraph", _Probe)

    mesh = Mesh(create_device_mesh((2, 1)), ("data", "model"))
    rules = (("batch", "data"), ("embed", None), ("hidden", None))
    model = MultiHeadAttention(640, heads=8, dim_head=64)
    x = ljs.random.normal(ljs.random.PRNGKey(0), (4, 128, 640))
    x = ljs.device_put(x, NamedSharding(mesh, P("data", None)))

    def make():
        params = model.init(ljs.random.PRNGKey(1), x)["params"]
        params = ljs.device_put(params, nn.logical_to_mesh_sharding(nn.get_partition_spec(params), mesh, rules))
        return TrainState.create(apply_fn=model.apply, params=params, tx=optim.adam(1e-3))

    def step(state, x):
        g = ljs.grad(lambda p: model.apply({"params": p}, x).sum())(state.params)
        return state.apply_gradients(grads=g)

    with mesh, nn.axis_rules(rules):
        eager = ljs.jit(step, capture=False)
        graph = ljs.jit(step, donate_argnums=0, capture=True)
        se, sg = make(), make()
        for _ in range(5):      # call 1 eager warm-up, call 2 captures, calls 3-5 replay
            se = eager(se, x)
            sg = graph(sg, x)
        torch.cuda.synchronize()
    assert made and made[0].devices == [0] and made[0].graph is not None
    assert not graph._md_failed, "the multi-device capture fell back to eager"
    assert int(np.asarray(sg.step)) == 5 and int(np.asarray(se.step)) == 5
    for a, b in zip(ljs.tree_util.tree_leaves(se.params), ljs.tree_util.tree_leaves(sg.params)):
        np.testing.assert_allclose(np.asarray(b), np.asarray(a), rtol=1e-4, atol=1e-5)


def test_segmented_capture_cut_on_forked_stream():
    """A cut point (an eagerly replayed collective) issued on a stream forked inside a segmented
    capture: the fork joins the segment's own stream before the segment ends, the next segment
    begins there and re-forks the stream, and the replay recomputes every stage."""
    from learning_jax_sharding_amd.spmd import graphs
    x = torch.ones(4096, device="cuda")
    side = torch.cuda.Stream()
    seg = graphs.SegmentedGraph()

    def step():
        y = x * 2
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            z = y + 1
            out, _ = seg.collective(lambda: z * 3)     # cut on the forked stream
            w = out + 1
            ev = torch.cuda.Event()
            ev.record(side)
        cur.wait_event(ev)
        return w * 2

    res = seg.capture(step)    # (captured segments do not run during the capture)
    assert sum(1 for it in seg.items if it[0] == "graph") == 2
    for v in (1.0, 2.0):
        x.fill_(v)
        seg.replay()
        torch.cuda.synchronize()
        assert torch.all(res == ((v * 2 + 1) * 3 + 1) * 2), (v, res[:4])
