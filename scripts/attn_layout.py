"""Attention fwd+bwd time by activation layout (the 2-D layout's local shapes: 128 sequences,
128 local queries, 256 gathered keys): batch-major vs seq-major storage vs seq-major with the
sequence stride padded off a power of two.

usage: python scripts/attn_layout.py [B Sq Sk] [ITERS]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402

B, Sq, Sk = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (128, 128, 256)
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
H, D = 8, 64


def make(S, layout):
    if layout == "batch":
        return torch.randn(B, S, H, D, device="cuda").bfloat16()
    pad = 64 if layout == "seqpad" else 0
    base = torch.randn(S, B * H * D + pad, device="cuda").bfloat16()
    return base[:, :B * H * D].view(S, B, H, D).permute(1, 0, 2, 3)


for layout in ("batch", "seq", "seqpad"):
    q = make(Sq, layout).requires_grad_()
    k = make(Sk, layout).requires_grad_()
    v = make(Sk, layout).requires_grad_()
    g = torch.randn(B, Sq, H, D, device="cuda").bfloat16()
    for _ in range(3):
        o = hip.attention(q, k, v, 0.125)
        torch.autograd.grad(o, (q, k, v), g)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for _ in range(iters):
        e[0].record()
        o = hip.attention(q, k, v, 0.125)
        e[1].record()
        torch.autograd.grad(o, (q, k, v), g)
        e[2].record()
        torch.cuda.synchronize()
        tf += e[0].elapsed_time(e[1])
        tb += e[1].elapsed_time(e[2])
    print(f"{layout:7s} B={B} Sq={Sq} Sk={Sk}: fwd {tf / iters * 1e3:.1f} us  bwd {tb / iters * 1e3:.1f} us", flush=True)
