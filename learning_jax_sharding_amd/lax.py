"""``jax.lax`` subset (``jax.lax.dot`` at ``case1a.py:49``)."""
from .ops.core import (  # noqa: F401
    convert as convert_element_type,
    dot,
    dot_general,
    reduce_max,
    reduce_sum,
    reshape,
    transpose,
    with_sharding_constraint,
)
from .ops.core import concatenate, softmax  # noqa: F401
