"""learning_jax_sharding_amd - an MI355X-native SPMD sharding framework.

A PyTorch-ROCm re-design of the capabilities of ``entrpn/learning-jax-sharding``
(JAX GSPMD case studies): Mesh / PositionalSharding / NamedSharding /
PartitionSpec / with_sharding_constraint over global-view sharded arrays, an
eager partitioner that lowers annotated ops to RCCL all-gather /
reduce-scatter / all-reduce / all-to-all over xGMI, hand-written CDNA4 HIP
kernels (MFMA GEMMs, fused attention, Adam, Philox RNG) and HIP-graph replay
in place of a tracing compiler.

The public surface mirrors the JAX modules the reference imports, so the case
studies read the same::

    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd.experimental import mesh_utils
    from learning_jax_sharding_amd.sharding import PositionalSharding
"""
from . import dtypes  # noqa: F401
from .runtime.devices import (  # noqa: F401
    Device, default_backend, device_count, devices, initialize_distributed, local_device_count,
    local_devices, process_count, process_index,
)
from .mesh import Mesh  # noqa: F401
from .array import ShapeDtypeStruct, Shard, ShardedArray, device_put  # noqa: F401
from .array import ShardedArray as Array  # noqa: F401
from .sharding import (  # noqa: F401
    GSPMDSharding, NamedSharding, PartitionSpec, PositionalSharding, SingleDeviceSharding,
)
from .spmd.api import eval_shape, grad, jit, value_and_grad  # noqa: F401
from .ops.core import with_sharding_constraint  # noqa: F401
from . import debug, experimental, lax, ops, random, tree_util  # noqa: F401
from . import nn, optim, training, models  # noqa: F401
from . import numpy  # noqa: F401
from . import parallel, profiler  # noqa: F401
from .utils import checkpoint  # noqa: F401
from .utils.tree import tree_map, tree_leaves, tree_flatten, tree_unflatten  # noqa: F401


def block_until_ready(x):
    for leaf in tree_leaves(x, is_leaf=lambda a: isinstance(a, ShardedArray)):
        if isinstance(leaf, ShardedArray):
            leaf.block_until_ready()
    return x


__version__ = "0.1.0"
