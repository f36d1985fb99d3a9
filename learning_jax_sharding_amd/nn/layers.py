"""Layers: Dense, Dropout, FeedForward, activations.

``Dense`` follows flax semantics (``case6_attention.py:61-90``): kernel
``(in, out)`` in ``param_dtype`` (f32), inputs/kernel/bias promoted to
``dtype`` (bf16) for the matmul, bias default on.  The matmul is the fused
MFMA GEMM with a bias epilogue (:func:`..ops.core.dense`).
"""
from __future__ import annotations

from typing import Any, Callable, Optional, Sequence, Tuple

import torch

from .. import dtypes as _dt
from ..array import ShardedArray
from ..ops import core
from . import initializers as init
from .module import Module, compact
from .partitioning import with_logical_constraint, with_logical_partitioning

__all__ = ["Dense", "DenseGeneral", "Dropout", "FeedForward", "relu", "gelu", "softmax", "Embed", "LayerNorm"]


def relu(x):
    return core.unary("relu", x)


def gelu(x):
    return core.binary("mul", x, core.unary("sigmoid", core.binary("mul", x, 1.702)))


def softmax(x, axis: int = -1):
    return core.softmax(x, axis)


class Dense(Module):
    features: int
    use_bias: bool = True
    dtype: Any = None
    param_dtype: Any = torch.float32
    precision: Any = None
    kernel_init: Callable = init.lecun_normal()
    bias_init: Callable = init.zeros

    def kernel_param(self, in_features: int) -> ShardedArray:
        return self.param("kernel", self.kernel_init, (in_features, self.features),
                          _dt.canonicalize(self.param_dtype))

    def bias_param(self) -> Optional[ShardedArray]:
        if not self.use_bias:
            return None
        return self.param("bias", self.bias_init, (self.features,), _dt.canonicalize(self.param_dtype))

    def __call__(self, inputs: ShardedArray, residual: Optional[ShardedArray] = None,
                 kernel: Optional[ShardedArray] = None) -> ShardedArray:
        """``inputs @ kernel (+ bias)``; ``residual`` is added in the compute dtype (fused into the
        GEMM epilogue on the MFMA path).  ``kernel``: this layer's kernel already gathered (an FSDP
        prefetch, parallel/fsdp.py) in place of the parameter."""
        if kernel is None:
            kernel = self.kernel_param(inputs.shape[-1])
        bias = self.bias_param()
        dtype = _dt.canonicalize(self.dtype) or _dt.result_type(inputs.dtype, kernel.dtype)
        return core.dense(inputs, [kernel], bias, compute_dtype=dtype, residual=residual)[0]


DenseGeneral = Dense


class Dropout(Module):
    """``nn.Dropout`` (``case6_attention.py:91,143``): identity when deterministic or rate 0; else
    keep-mask from the Philox uniform of each element's global index (mesh-invariant), kept values
    divided by the keep probability - one fused HIP kernel per shard on GPU (``hip.dropout``)."""

    rate: float = 0.0
    deterministic: Optional[bool] = None

    def __call__(self, x: ShardedArray, deterministic: Optional[bool] = None, rng=None) -> ShardedArray:
        det = self.deterministic if deterministic is None else deterministic
        if det or self.rate == 0.0:
            return x
        from .. import random as _random
        k = rng if rng is not None else self.make_rng("dropout")
        keep = 1.0 - self.rate
        if x.local and all(t.is_cuda and t.dtype in (torch.float32, torch.bfloat16) for t in x.local.values()):
            # one fused HIP pass per shard: the Philox uniform of each element's global index (the
            # draw of random.uniform below, bit for bit), compare, scale; the backward recomputes
            # the mask from the key instead of storing it
            from ..ops import hip
            loc = {d: hip.dropout(t, x.shape, x.tile.region(d, x.shape), k.k0, k.k1, keep)
                   for d, t in x.local.items()}
            return ShardedArray(x.shape, x.dtype, x.sharding, loc)
        u = _random.uniform(k, x.shape, torch.float32, sharding=x.sharding)
        scaled = core.binary("div", x, keep)
        return core.where(_lt(u, keep), scaled, 0.0)


def _lt(u: ShardedArray, v: float) -> ShardedArray:
    return ShardedArray(u.shape, torch.bool, u.sharding, {d: t < v for d, t in u.local.items()})


class FeedForward(Module):
    """``y = relu(x Win) Wout`` - the FF layer of the reference's comments (``case6_attention.py:36-40``).

    Logical axes ``Win: ('embed','hidden')``, ``Wout: ('hidden','embed')`` so the
    declared rule ``('hidden','model')`` (``case6_attention.py:186``) shards the
    hidden dim Megatron-style.  ``fp8=True`` runs the GEMMs on CDNA4's MX-fp8 block-scaled MFMA
    (e4m3 elements, e8m0 scales per 32 elements along K): with replicated weights the fused
    block of :func:`ops.fp8.ff_block`, with the hidden dim split over a device group the
    tensor-parallel fused block :func:`ops.fp8.ff_block_tp` (every FF GEMM in fp8 either way);
    any other layout runs the two forward GEMMs in fp8 with a bf16 backward.
    """

    hidden_dim: int
    dtype: Any = torch.bfloat16
    fp8: bool = False

    @compact
    def __call__(self, x: ShardedArray, residual: Optional[ShardedArray] = None) -> ShardedArray:
        """``residual`` (e.g. ``x`` itself for a skip connection) is added to the output in the
        compute dtype, fused into the down projection's GEMM epilogue."""
        d = x.shape[-1]
        w_in = self.param("w_in", with_logical_partitioning(init.lecun_normal(), ("embed", "hidden")),
                          (d, self.hidden_dim), torch.float32)
        w_out = self.param("w_out", with_logical_partitioning(init.lecun_normal(), ("hidden", "embed")),
                           (self.hidden_dim, d), torch.float32)
        dt = _dt.canonicalize(self.dtype)
        loc = next(iter(x.local.values())) if x.local else None
        tokens_ok = loc is not None and (loc.numel() // max(1, d)) % 128 == 0
        # weights not split along the hidden dim (replicated, or only M split - the reference
        # rules map 'embed' before 'hidden', case6_attention.py:183-187): gathered, and every
        # device runs the fused block on its own tokens (no activation moves)
        hidden_split = w_in.tile.tile_shape[1] > 1 or w_out.tile.tile_shape[0] > 1
        if dt == torch.bfloat16 and not hidden_split and (residual is None or residual is x) \
                and (d % 128 == 0 and self.hidden_dim % 128 == 0 and tokens_ok if self.fp8 else True):
            # replicated weights (data-parallel / single device): the fused block - one autograd
            # node, epilogue fusions across its GEMMs; fp8: every FF GEMM (forward, dX and the
            # weight gradients) on MX-fp8, the hidden activation stored only as MX-fp8, the
            # quantized operands written by their producers' epilogues
            from ..ops.fp8 import ff_block
            return ff_block(x, w_in, w_out, residual=residual, fp8=self.fp8)
        if dt == torch.bfloat16 and (d % 128 == 0 and self.hidden_dim % 128 == 0 if self.fp8 else True):
            # the hidden dim split over a device group (rule ('hidden', 'model')): the
            # tensor-parallel fused block - x's token blocks gathered over the group, W_in
            # column- / W_out row-parallel, the partial outputs reduce-scattered (fp8: every FF
            # GEMM on the MX MFMA, as in the replicated case)
            from ..ops.fp8 import ff_block_tp, ff_block_tp_plan
            xg = x
            if x.tile.tile_shape[-1] > 1:
                from ..spmd.reshard import reshard_tile
                xg = reshard_tile(x, x.tile.unshard([x.ndim - 1]), note="ff.x")
            plan = ff_block_tp_plan(xg, w_in, w_out)
            tp = len(plan[0][0]) if plan is not None else 1
            if plan is not None and self._tp_tokens_ok(xg, plan) and (
                    not self.fp8 or (self.hidden_dim // tp) % 128 == 0):
                return ff_block_tp(xg, w_in, w_out, residual=residual, fp8=self.fp8, plan=plan)
        if self.fp8:
            from ..ops.fp8 import fp8_dense
            h = fp8_dense(x, w_in, relu=True, out_dtype=dt)
            h = with_logical_constraint(h, ("batch", "length", "hidden"))
            y = fp8_dense(h, w_out, relu=False, out_dtype=dt)
            return y if residual is None else core.binary("add", core.convert(residual, dt), y)
        h = core.dense(x, [w_in], None, compute_dtype=dt, relu=True)[0]
        h = with_logical_constraint(h, ("batch", "length", "hidden"))
        return core.dense(h, [w_out], None, compute_dtype=dt, residual=residual)[0]


    @staticmethod
    def _tp_tokens_ok(x: ShardedArray, plan) -> bool:
        """The gathered token count per device is a multiple of 128 (the MX weight gradients
        contract over tokens in 128-deep K-tiles)."""
        groups, k = plan
        loc = next(iter(x.local.values()), None)
        if loc is None:
            return False
        return (loc.numel() // max(1, x.shape[-1]) * len(groups[0])) % 128 == 0


class Embed(Module):
    num_embeddings: int
    features: int
    param_dtype: Any = torch.float32

    def __call__(self, ids: ShardedArray) -> ShardedArray:
        table = self.param("embedding", init.normal(1.0), (self.num_embeddings, self.features),
                           _dt.canonicalize(self.param_dtype))
        # rows gathered locally: the table is replicated onto the ids' devices first
        from ..sharding.tile import TileAssignment
        from ..spmd.reshard import reshard_tile
        tab = reshard_tile(table, TileAssignment.replicated(ids.tile.device_ids, 2))
        loc = {d: tab.local[d][ids.local[d].long()] for d in ids.local}
        tile = ids.tile.insert_dims(list(range(ids.ndim)), ids.ndim + 1)
        from ..sharding.shardings import sharding_from_tile
        return ShardedArray(tuple(ids.shape) + (self.features,), table.dtype,
                            sharding_from_tile(tile, like=[ids.sharding]), loc)


class LayerNorm(Module):
    epsilon: float = 1e-6
    dtype: Any = None
    use_bias: bool = True
    use_scale: bool = True

    def __call__(self, x: ShardedArray) -> ShardedArray:
        d = x.shape[-1]
        scale = self.param("scale", init.ones, (d,), torch.float32) if self.use_scale else None
        bias = self.param("bias", init.zeros, (d,), torch.float32) if self.use_bias else None
        xf = core.convert(x, torch.float32)
        mean = core.reduce_mean(xf, -1, keepdims=True)
        xc = core.binary("sub", xf, mean)
        var = core.reduce_mean(core.binary("mul", xc, xc), -1, keepdims=True)
        y = core.binary("mul", xc, core.unary("rsqrt", core.binary("add", var, self.epsilon)))
        if scale is not None:
            y = core.binary("mul", y, scale)
        if bias is not None:
            y = core.binary("add", y, bias)
        return core.convert(y, _dt.canonicalize(self.dtype) or x.dtype)
