"""Local (per-shard) optimizer kernels: fused Adam on HIP, torch on host devices."""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .kernels import use_hip

__all__ = ["adam_fused", "adam_moments_and_update"]


def _torch_adam(p, g, m, v, step, lr, b1, b2, eps, wd):
    s = step.to(torch.float32)
    bc1 = 1.0 - torch.pow(torch.tensor(b1, dtype=torch.float32, device=s.device), s)
    bc2 = 1.0 - torch.pow(torch.tensor(b2, dtype=torch.float32, device=s.device), s)
    gf = g.to(torch.float32)
    m2 = b1 * m + (1.0 - b1) * gf
    v2 = b2 * v + (1.0 - b2) * gf * gf
    upd = (m2 / bc1) / (torch.sqrt(v2 / bc2) + eps)
    if wd:
        upd = upd + wd * p
    return -lr * upd, m2, v2


def adam_fused(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: torch.Tensor,
               lr: float, b1: float, b2: float, eps: float, wd: float = 0.0, inplace: bool = False
               ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """One fused pass: returns (p', m', v'); writes into p/m/v when ``inplace``."""
    if use_hip(p):
        from . import hip
        return hip.adam(p, g, m, v, step, lr, b1, b2, eps, wd, inplace)
    with torch.no_grad():
        u, m2, v2 = _torch_adam(p, g, m, v, step, lr, b1, b2, eps, wd)
        if inplace:
            p.add_(u.to(p.dtype))
            m.copy_(m2)
            v.copy_(v2)
            return p, m, v
        return (p + u).to(p.dtype), m2, v2


def adam_moments_and_update(g, m, v, step, lr, b1, b2, eps, p: Optional[torch.Tensor] = None, wd: float = 0.0):
    with torch.no_grad():
        return _torch_adam(p if p is not None else torch.zeros_like(g), g, m, v, step, lr, b1, b2, eps, wd)
