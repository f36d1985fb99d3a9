"""``jax.sharding`` equivalent."""
from ..mesh import Mesh  # noqa: F401
from .shardings import (  # noqa: F401
    GSPMDSharding,
    NamedSharding,
    P,
    PartitionSpec,
    PositionalSharding,
    ReplicatedSharding,
    default_sharding,
    Sharding,
    SingleDeviceSharding,
    sharding_from_tile,
)
from .tile import TileAssignment  # noqa: F401
