"""``jax.tree_util`` subset."""
from .utils.tree import (  # noqa: F401
    register_pytree_node, tree_flatten, tree_leaves, tree_map, tree_structure, tree_unflatten,
)
