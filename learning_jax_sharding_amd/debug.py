"""``jax.debug`` subset."""
from .utils.visualize import visualize_array_sharding, visualize_sharding  # noqa: F401
