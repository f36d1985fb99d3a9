"""Global-view ops (partitioned) and their per-device kernels."""
from .core import (  # noqa: F401
    binary, concatenate, convert, dense, dot, dot_general, dot_product_attention, einsum, getitem, matmul,
    reduce_max, reduce_mean, reduce_sum, reshape, softmax, transpose, unary, with_sharding_constraint,
)
