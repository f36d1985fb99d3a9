"""``flax.linen`` equivalent (modules, layers, logical-axis partitioning)."""
from . import initializers  # noqa: F401
from . import partitioning  # noqa: F401
from .layers import Dense, DenseGeneral, Dropout, Embed, FeedForward, LayerNorm, gelu, relu, softmax  # noqa: F401
from .module import Module, Scope, compact  # noqa: F401
from .partitioning import (  # noqa: F401
    LogicallyPartitioned, Partitioned, axis_rules, get_partition_spec, logical_to_mesh, logical_to_mesh_axes,
    logical_to_mesh_sharding, unbox, with_logical_constraint, with_logical_partitioning,
)
