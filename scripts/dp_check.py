"""Data-parallel train-step check: run K steps of the case6 block and save the parameters.

Launched with torchrun (one rank per device; ``LJS_DIST_BACKEND=gloo`` lets several ranks
share one GPU) or as a single process (the reference).  The global batch is fixed, so every
world size must reach the same parameters.  Used by ``tests/test_distributed_gpu.py``.

usage: python scripts/dp_check.py OUT.npz STEPS CAPTURE(0/1) [GLOBAL_BATCH] [MESH DxM]

With MESH (e.g. 1x2 or 2x2) the reference's 2-D layout runs: sequence over 'model', Q/K/V
weights sharded over 'model' (case6_attention.py:155-162,183-187).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _log(msg):
    print(f"[rank {os.environ.get('RANK', '0')}] {msg}", file=sys.stderr, flush=True)


def main():
    if os.environ.get("LJS_HANG_DUMP_S"):
        import faulthandler
        faulthandler.dump_traceback_later(int(os.environ["LJS_HANG_DUMP_S"]), exit=True)
    out, steps, capture = sys.argv[1], int(sys.argv[2]), sys.argv[3] == "1"
    gb = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1:
        os.environ.setdefault("LJS_NUM_DEVICES", "1")
    import numpy as np
    import torch
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd import nn, optim
    from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh
    from learning_jax_sharding_amd.models import MultiHeadAttention
    from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P
    from learning_jax_sharding_amd.training import TrainState

    n = ljs.device_count()
    mshape = tuple(int(v) for v in sys.argv[5].split("x")) if len(sys.argv) > 5 and world > 1 else (n, 1)
    assert mshape[0] * mshape[1] == n, (mshape, n)
    mesh = Mesh(create_device_mesh(mshape), ("data", "model"))
    rules = (("batch", "data"), ("embed", "model"), ("hidden", "model"))
    model = MultiHeadAttention(640, heads=8, dim_head=64)
    xs = NamedSharding(mesh, P("data", "model"))
    x = ljs.random.normal(ljs.random.PRNGKey(0), (gb, 128, 640), sharding=xs)

    def init_fn(k, x):
        return TrainState.create(apply_fn=model.apply, params=model.init(k, x)["params"], tx=optim.adam(1e-3))

    abstract = ljs.eval_shape(init_fn, ljs.random.PRNGKey(1), x)
    ss = nn.logical_to_mesh_sharding(nn.get_partition_spec(abstract), mesh, rules)
    state = ljs.jit(init_fn, out_shardings=ss)(ljs.random.PRNGKey(1), x)
    _log(f"initialised on {n} devices")

    def train_step(state, x):
        g = ljs.grad(lambda p: model.apply({"params": p}, x).sum())(state.params)
        return state.apply_gradients(grads=g)

    # LJS_CHECK_MULTI=G: G steps per jitted call, each registering the next step's input as
    # bench.py does (ops/linear.prefetch_next_input: the early input cast)
    G = int(os.environ.get("LJS_CHECK_MULTI", "1"))
    if G > 1:
        from learning_jax_sharding_amd.ops import linear as _lin

        def train_steps(state, x):
            for i in range(G):
                if i + 1 < G:
                    _lin.prefetch_next_input(x)
                state = train_step(state, x)
            _lin.join_precasts()
            return state
        step = ljs.jit(train_steps, in_shardings=(ss, xs), out_shardings=ss, donate_argnums=0, capture=capture)
        assert steps % G == 0, (steps, G)
        steps //= G
    else:
        step = ljs.jit(train_step, in_shardings=(ss, xs), out_shardings=ss, donate_argnums=0, capture=capture)
    with mesh, nn.axis_rules(rules):
        for i in range(steps):
            state = step(state, x)
            _log(f"step {i} issued")
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    leaves = ljs.tree_util.tree_leaves(nn.unbox(state.params))
    # np.asarray of a global array is a collective in multi-process runs: every rank calls it
    arrs = [np.asarray(l) for l in leaves]
    stp = np.asarray(state.step)
    _log("gathered")
    if int(os.environ.get("RANK", "0")) == 0:
        extra = {}
        if G > 1:
            extra["precast_taken"] = np.asarray(_lin.PRECAST_STATS["taken"])
        np.savez(out, *arrs, step=stp, **extra)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
