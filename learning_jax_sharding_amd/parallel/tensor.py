"""Tensor (model) parallelism: logical-axis rule presets and explicit column/row-parallel
dense layers.

The reference's "model" axis shards the attention weights on their *contraction* dim
(``('embed', 'model')``, ``case6_attention.py:185``; heads deliberately replicated,
``case6_attention.py:101-103``) and the activations on the *sequence* dim, so GSPMD
gathers the weights before the QKV projections and all-to-alls the out-projection
(SURVEY §2.7).  That plan is reproduced by the partitioner from ``REFERENCE_RULES``.

``GSPMD2D_RULES`` (preset ``"gspmd2d"``) is the GSPMD paper's "2D finalized" attention layout
the reference's comment names (``case6_attention.py:53-55``: "MND ... Shardings: X,Y,_"):
``embed -> data``, ``heads -> model``, so Wq/Wk/Wv are split over BOTH mesh axes - (320, 256)
per device on the 2x2 mesh, the shape the stale comment at ``case6_attention.py:222-227``
expects.

``MEGATRON_RULES`` (preset ``"megatron"``) shards heads and the FF hidden dim over ``model``
and keeps ``embed`` replicated (column-parallel QKV / W_in, row-parallel W_out / W_o, one
all-reduce per block in forward and one in backward) - on 8 xGMI-connected MI355X this
moves far fewer bytes per step than gathering weights and sequence, so it is the preferred
TP layout there.

:func:`column_parallel` / :func:`row_parallel` are the explicit Megatron building blocks on
global-view arrays: they pin the shardings, and the partitioner lowers the matmul with
the collective the layout implies (none / all-reduce or reduce-scatter).
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

from ..array import ShardedArray
from ..mesh import Mesh, current_mesh
from ..ops import core
from ..sharding import NamedSharding, PartitionSpec as P

__all__ = ["REFERENCE_RULES", "FSDP_RULES", "GSPMD2D_RULES", "MEGATRON_RULES", "DP_RULES", "PRESETS", "rules", "column_parallel",
           "row_parallel"]

Rules = Tuple[Tuple[str, Optional[str]], ...]

# case6_attention.py:183-187
REFERENCE_RULES: Rules = (("batch", "data"), ("embed", "model"), ("hidden", "model"))
# case5_attention_dense.py:109-112: embed on data (FSDP-style weight sharding)
FSDP_RULES: Rules = (("batch", "data"), ("embed", "data"), ("kv", None), ("hidden", "model"))
# GSPMD paper "2D finalized" (case6_attention.py:53-55): weights split over data AND model
GSPMD2D_RULES: Rules = (("batch", "data"), ("embed", "data"), ("heads", "model"), ("hidden", "model"))
# heads / FF hidden over model, batch over data, embed replicated
MEGATRON_RULES: Rules = (("batch", "data"), ("heads", "model"), ("hidden", "model"), ("embed", None),
                         ("kv", None), ("length", None))
# pure data parallelism (every weight replicated)
DP_RULES: Rules = (("batch", "data"),)

PRESETS = {"reference": REFERENCE_RULES, "case6": REFERENCE_RULES, "fsdp": FSDP_RULES, "case5": FSDP_RULES,
           "gspmd2d": GSPMD2D_RULES, "megatron": MEGATRON_RULES, "dp": DP_RULES}


def rules(name: str) -> Rules:
    try:
        return PRESETS[name]
    except KeyError:
        raise ValueError(f"unknown rules preset {name!r}; have {sorted(PRESETS)}") from None


def _mesh(mesh: Optional[Mesh]) -> Mesh:
    m = mesh or current_mesh()
    if m is None:
        raise ValueError("tensor-parallel layers need a mesh (argument or `with mesh:`)")
    return m


def column_parallel(x: ShardedArray, w: ShardedArray, b: Optional[ShardedArray] = None, axis: str = "model",
                    batch_axis: Optional[str] = "data", gather_output: bool = False, relu: bool = False,
                    compute_dtype=None, mesh: Optional[Mesh] = None) -> ShardedArray:
    """``y = x @ w (+b)`` with ``w`` split on its OUTPUT features over ``axis``: every shard
    computes its own column block, no communication; ``gather_output`` all-gathers y."""
    m = _mesh(mesh)
    lead = [batch_axis] + [None] * (x.ndim - 2)
    x = core.with_sharding_constraint(x, NamedSharding(m, P(*lead, None)))
    w = core.with_sharding_constraint(w, NamedSharding(m, P(None, axis)))
    if b is not None:
        b = core.with_sharding_constraint(b, NamedSharding(m, P(axis)))
    y = core.dense(x, [w], b, compute_dtype=compute_dtype, relu=relu)[0]
    if gather_output:
        y = core.with_sharding_constraint(y, NamedSharding(m, P(*lead, None)))
    return y


def row_parallel(x: ShardedArray, w: ShardedArray, b: Optional[ShardedArray] = None, axis: str = "model",
                 batch_axis: Optional[str] = "data", scatter_dim: Optional[int] = None, compute_dtype=None,
                 mesh: Optional[Mesh] = None) -> ShardedArray:
    """``y = x @ w (+b)`` with ``w`` split on its INPUT features over ``axis`` (x arrives
    column-split from a :func:`column_parallel` layer): partial products are all-reduced,
    or reduce-scattered along ``scatter_dim`` (sequence parallelism) when given."""
    m = _mesh(mesh)
    lead = [batch_axis] + [None] * (x.ndim - 2)
    x = core.with_sharding_constraint(x, NamedSharding(m, P(*lead, axis)))
    w = core.with_sharding_constraint(w, NamedSharding(m, P(axis, None)))
    y = core.dense(x, [w], b, compute_dtype=compute_dtype)[0]
    if scatter_dim is not None:
        spec = [batch_axis] + [None] * (y.ndim - 1)
        spec[scatter_dim] = axis
        y = core.with_sharding_constraint(y, NamedSharding(m, P(*spec)))
    return y
