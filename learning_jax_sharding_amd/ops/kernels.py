"""Per-device compute: hand-written HIP kernels on MI355X, torch on host devices.

Every function here takes and returns *local* torch tensors (one device's
shard).  On a ROCm tensor the call goes to the gfx950 HIP extension
(:mod:`.hip`); that path fails loudly if the extension is not built - there
is no silent torch fallback for GPU tensors (``LJS_ALLOW_TORCH_FALLBACK=1``
opts in, for debugging only).  Host-device (CPU) tensors use torch, which is
also the numerical oracle the GPU tests compare against.

Numerics follow the reference's bf16 recipe (``case6_attention.py:46,120-130``):
bf16 operands, f32 accumulation, f32 softmax, probabilities rounded to bf16
before P·V.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import torch

__all__ = ["cast", "reduce_sum", "dot_general", "linear", "softmax", "attention", "use_hip"]

_LOW = (torch.bfloat16, torch.float16)


def use_hip(t: torch.Tensor) -> bool:
    return t.is_cuda and not t.is_meta


def _hip():
    from . import hip
    return hip


# ----------------------------------------------------------------------------- casts / reductions
def cast(t: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    if t.dtype == dtype:
        return t
    if use_hip(t) and _hip().supports_cast(t.dtype, dtype):
        return _hip().cast(t, dtype)
    return t.to(dtype)


def reduce_sum(t: torch.Tensor, axes: Sequence[int], keepdim: bool, acc_dtype: torch.dtype) -> torch.Tensor:
    if not axes:
        return t.to(acc_dtype)
    if use_hip(t) and len(axes) == t.dim() and not keepdim:
        return _hip().sum_all(t, acc_dtype)
    return t.sum(dim=tuple(axes), keepdim=keepdim, dtype=acc_dtype)


def mse_loss(y: torch.Tensor, t: torch.Tensor, scale: float) -> torch.Tensor:
    """``scale * sum((y - t)^2)`` of one shard in f32 (fused HIP pass with its gradient on GPU)."""
    if use_hip(y):
        return _hip().mse_loss(y, t, scale)
    return ((y.float() - t.float()) ** 2).sum() * scale


# ----------------------------------------------------------------------------- matmuls
def _to_bmk(a: torch.Tensor, batch, free, contract):
    perm = list(batch) + list(free) + list(contract)
    x = a.permute(perm)
    B = 1
    for i in batch:
        B *= a.shape[i]
    M = 1
    for i in free:
        M *= a.shape[i]
    Kd = 1
    for i in contract:
        Kd *= a.shape[i]
    return x.reshape(B, M, Kd)


def dot_general(a: torch.Tensor, b: torch.Tensor, lc, rc, lb, rb, out_dtype: torch.dtype) -> torch.Tensor:
    lf = [i for i in range(a.dim()) if i not in lc and i not in lb]
    rf = [i for i in range(b.dim()) if i not in rc and i not in rb]
    A = _to_bmk(a, lb, lf, lc)                       # (B, M, K)
    Bt = _to_bmk(b, rb, rf, rc)                      # (B, N, K)
    out_shape = [a.shape[i] for i in lb] + [a.shape[i] for i in lf] + [b.shape[i] for i in rf]
    if use_hip(a):
        C = _hip().bmm_nt(A, Bt, out_dtype)          # C[b] = A[b] @ Bt[b]^T
    else:
        if A.dtype in _LOW or Bt.dtype in _LOW:
            C = torch.bmm(A.float(), Bt.float().transpose(1, 2)).to(out_dtype)
        else:
            C = torch.bmm(A.to(out_dtype if out_dtype.is_floating_point else A.dtype),
                          Bt.to(out_dtype if out_dtype.is_floating_point else Bt.dtype).transpose(1, 2)).to(out_dtype)
    return C.reshape(out_shape)


def linear(x: torch.Tensor, ws: Sequence[torch.Tensor], b: Optional[torch.Tensor], compute_dtype: torch.dtype,
           relu: bool = False, out_dtype: Optional[torch.dtype] = None, fp8: bool = False,
           residual: Optional[torch.Tensor] = None) -> List[torch.Tensor]:
    """``[x @ w (+ b)(relu) for w in ws]`` in ``compute_dtype`` (flax ``Dense`` semantics);
    ``fp8`` = MX-fp8 forward GEMMs (HIP block-scaled MFMA, exact emulation on CPU).
    ``residual`` (one kernel): ``out + residual`` in the output dtype, both operands rounded to
    it first (the GPU fuses the add into the GEMM epilogue)."""
    out_dtype = out_dtype or compute_dtype
    if fp8:
        from . import fp8 as F8
        outs = [F8.linear_fp8(x, w, b, relu, out_dtype) for w in ws]
        if residual is not None:
            outs[0] = outs[0] + residual.to(outs[0].dtype)
        return outs
    if use_hip(x):
        return _hip().linear(x, list(ws), b, compute_dtype, relu, out_dtype, residual=residual)
    if residual is not None:
        outs = linear(x, ws, b, compute_dtype, relu, out_dtype)
        return [outs[0] + residual.to(outs[0].dtype)] + outs[1:]
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    xc = x2.to(compute_dtype)
    outs = []
    for w in ws:
        wc = w.to(compute_dtype)
        if compute_dtype in _LOW:
            y = xc.float() @ wc.float()
            if b is not None:
                y = y + b.to(compute_dtype).float()
        else:
            y = xc @ wc
            if b is not None:
                y = y + b.to(compute_dtype)
        if relu:
            y = torch.relu(y)
        outs.append(y.to(out_dtype).reshape(tuple(lead) + (w.shape[-1],)))
    return outs


# ----------------------------------------------------------------------------- softmax / attention
def softmax(t: torch.Tensor, axis: int) -> torch.Tensor:
    if use_hip(t) and axis % t.dim() == t.dim() - 1 and t.dtype == torch.float32:
        return _hip().softmax_lastdim(t)
    return torch.softmax(t.float(), dim=axis).to(t.dtype)


def attention_reference(q, k, v, scale: float, causal: bool = False, q_offset: int = 0) -> torch.Tensor:
    """Plain torch oracle of ``case6_attention.py:120-133`` on (b, s, n, h) tensors."""
    qf, kf = q.float(), k.float()
    s = torch.einsum("btnh,bfnh->bnft", kf, qf) * scale
    if causal:
        sq, sk = q.shape[1], k.shape[1]
        qi = torch.arange(sq, device=q.device)[:, None] + q_offset
        ki = torch.arange(sk, device=q.device)[None, :]
        s = s.masked_fill(ki > qi, float("-inf"))
    p = torch.softmax(s, dim=-1).to(v.dtype)
    o = torch.einsum("bnft,btnh->bfnh", p.float(), v.float())
    return o.to(v.dtype)


_WARNED_DH = set()


def _hip_attn(q, k, v) -> bool:
    """Whether the HIP attention kernels take these (b, s, heads, head_dim) operands: GPU tensors
    with head_dim 64 (the reference's, ``case6_attention.py``) contiguous in the last dim.  Other
    head dims run the torch formulation below on the GPU (same math, autograd through torch),
    with a one-time warning."""
    if not use_hip(q):
        return False
    if all(t.shape[-1] == 64 and t.stride(-1) == 1 for t in (q, k, v)):
        return True
    key = (q.shape[-1], v.shape[-1])
    if key not in _WARNED_DH:
        _WARNED_DH.add(key)
        import warnings
        warnings.warn(f"HIP attention kernels take head_dim 64; head_dim {q.shape[-1]} (v {v.shape[-1]}) runs "
                      "the torch attention formulation on the GPU")
    return False


def attention(q, k, v, scale: float, causal: bool = False, q_offset: int = 0) -> torch.Tensor:
    if _hip_attn(q, k, v):
        return _hip().attention(q, k, v, scale, causal, q_offset)
    return attention_reference(q, k, v, scale, causal, q_offset)


_LOG2E = 1.4426950408889634


def _block_scores(q, k, scale, causal, q_offset):
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) * scale
    if causal:
        Sq, Sk = q.shape[1], k.shape[1]
        qi = torch.arange(Sq, device=q.device)[:, None] + q_offset
        ki = torch.arange(Sk, device=q.device)[None, :]
        s = s.masked_fill(ki > qi, float("-inf"))
    return s


def attention_fwd_lse(q, k, v, scale: float, causal: bool = False, q_offset: int = 0):
    """One (q block, kv block) flash forward: (o normalised within the block, lse) with lse in
    the HIP kernels' convention - log2 of the scaled-score partition function, +inf for rows
    without any unmasked key."""
    if _hip_attn(q, k, v):
        return _hip().attn_fwd_lse(q, k, v, scale, causal, q_offset)
    s = _block_scores(q, k, scale, causal, q_offset)
    m = s.amax(-1, keepdim=True)
    empty = torch.isinf(m) & (m < 0)
    m = torch.where(empty, torch.zeros_like(m), m)
    p = torch.exp(s - m)
    l = p.sum(-1, keepdim=True)
    probs = (p / l.clamp(min=1e-30)).to(v.dtype).float()
    o = torch.einsum("bhqk,bkhd->bqhd", probs, v.float()).to(v.dtype)
    lse = ((m + torch.log(l)) * _LOG2E).squeeze(-1)
    lse = torch.where(empty.squeeze(-1), torch.full_like(lse, float("inf")), lse)
    return o, lse


def attention_fwd_merge(q, k, v, scale: float, causal: bool, q_offset: int, state, last: bool):
    """One key block of a blockwise forward merged into ``state`` = [o_acc f32, lse] (None before the
    first block).  On GPU the merge happens in the kernel's epilogue; ``last`` makes it write and
    return the final output in v's dtype (else returns None)."""
    if _hip_attn(q, k, v):
        B, Sq, H, D = q.shape
        if state[0] is None:
            state[0] = torch.empty((B, Sq, H, D), dtype=torch.float32, device=q.device)
            state[1] = torch.empty((B, H, Sq), dtype=torch.float32, device=q.device)
            mode = 1
        else:
            mode = 3 if last else 2
        if mode == 1 and last:
            # a single block: the plain forward (bf16 out + lse)
            o, lse = _hip().attn_fwd_lse(q, k, v, scale, causal, q_offset)
            state[1] = lse
            return o
        out = _hip().attn_fwd_acc(q, k, v, scale, causal, q_offset, state[0], state[1], mode)
        return out if last else None
    o_s, l_s = attention_fwd_lse(q, k, v, scale, causal, q_offset)
    if state[0] is None:
        state[0], state[1] = o_s.float(), l_s
    else:
        state[0], state[1] = _merge_lse(state[0], state[1], o_s, l_s)
    return state[0].to(v.dtype) if last else None


def _merge_lse(o, lse, o_s, lse_s):
    """Merge two partial attention results (o normalised per part, lse in log2; +inf = no keys)."""
    neg = torch.full_like(lse, float("-inf"))
    a = torch.where(torch.isinf(lse) & (lse > 0), neg, lse)
    b = torch.where(torch.isinf(lse_s) & (lse_s > 0), neg, lse_s)
    m = torch.maximum(a, b)
    m0 = torch.where(torch.isinf(m), torch.zeros_like(m), m)
    wa, wb = torch.exp2(a - m0), torch.exp2(b - m0)
    tot = wa + wb
    lse_new = torch.where(tot > 0, m0 + torch.log2(tot), torch.full_like(m, float("inf")))
    inv = torch.where(tot > 0, 1.0 / tot, torch.zeros_like(tot))
    ca = (wa * inv).permute(0, 2, 1)[..., None]
    cb = (wb * inv).permute(0, 2, 1)[..., None]
    return o.float() * ca + o_s.float() * cb, lse_new


def attention_bwd_block(q, k, v, o, do, lse, scale: float, causal: bool = False, q_offset: int = 0):
    """One kv block's (dq, dk, dv) given the final output ``o`` and global (log2) ``lse``."""
    if _hip_attn(q, k, v):
        return _hip().attn_bwd_block(q, k, v, o, do, lse, scale, causal, q_offset)
    s = _block_scores(q, k, scale, causal, q_offset)
    p = torch.exp(s - (lse / _LOG2E)[..., None])
    dof = do.float()
    dp = torch.einsum("bqhd,bkhd->bhqk", dof, v.float())
    delta = (dof * o.float()).sum(-1).permute(0, 2, 1)[..., None]       # [b,h,q,1]
    ds = p * (dp - delta)
    dq = torch.einsum("bhqk,bkhd->bqhd", ds, k.float()) * scale
    dk = torch.einsum("bhqk,bqhd->bkhd", ds, q.float()) * scale
    dv = torch.einsum("bhqk,bqhd->bkhd", p.to(v.dtype).float(), dof)
    return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype)
