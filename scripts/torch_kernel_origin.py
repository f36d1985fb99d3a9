"""Which Python-level op launched each GPU kernel of the bench train step (eager, no graph).

torch.profiler over two eager steps of the bench configuration; prints the ops sorted by
device time with their kernels, so stray torch kernels around the HIP ones can be traced
back to the code that launched them.  Usage: ``python scripts/torch_kernel_origin.py``.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("LJS_NUM_DEVICES", "1")

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import learning_jax_sharding_amd as ljs  # noqa: E402
from learning_jax_sharding_amd import nn, optim  # noqa: E402
from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh  # noqa: E402
from learning_jax_sharding_amd.models import MultiHeadAttention  # noqa: E402
from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P  # noqa: E402
from learning_jax_sharding_amd.training import TrainState  # noqa: E402


def main():
    B = int(os.environ.get("LJS_BENCH_BPG", "64"))
    mesh = Mesh(create_device_mesh((1, 1)), ("data", "model"))
    rules = (("batch", "data"), ("embed", "model"), ("hidden", "model"))
    model = MultiHeadAttention(640, heads=8, dim_head=64)
    xs = NamedSharding(mesh, P("data", "model"))
    x = ljs.random.normal(ljs.random.PRNGKey(0), (B, 256, 640), sharding=xs)

    def init_fn(k, x):
        return TrainState.create(apply_fn=model.apply, params=model.init(k, x)["params"], tx=optim.adam(1e-3))

    abstract = ljs.eval_shape(init_fn, ljs.random.PRNGKey(1), x)
    ss = nn.logical_to_mesh_sharding(nn.get_partition_spec(abstract), mesh, rules)
    state = ljs.jit(init_fn, out_shardings=ss)(ljs.random.PRNGKey(1), x)

    def train_step(state, x):
        g = ljs.grad(lambda p: model.apply({"params": p}, x).sum())(state.params)
        return state.apply_gradients(grads=g)

    step = ljs.jit(train_step, in_shardings=(ss, xs), out_shardings=ss, donate_argnums=0, capture=False)
    with mesh, nn.axis_rules(rules):
        for _ in range(3):
            state = step(state, x)
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                     with_stack=True) as prof:
            for _ in range(2):
                state = step(state, x)
            torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=45,
                                                              max_name_column_width=60))
    print(prof.key_averages(group_by_stack_n=6).table(sort_by="self_cuda_time_total", row_limit=25,
                                                       max_name_column_width=60))


if __name__ == "__main__":
    main()
