"""Run ONE attention kernel configuration repeatedly (for rocprofv3 counter passes).

usage: python scripts/attn_one.py {fwd,bwd} [B S H] [ITERS]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402

which = sys.argv[1]
B, S, H = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (64, 256, 8)
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
qkv = torch.randn(B, S, 3, H, 64, device="cuda").bfloat16()
q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
if which == "fwd":
    for _ in range(iters):
        hip.attention(q, k, v, 0.125)
else:
    q1, k1, v1 = (t.detach().requires_grad_() for t in (q, k, v))
    o = hip.attention(q1, k1, v1, 0.125)
    g = torch.randn_like(o)
    for _ in range(iters):
        torch.autograd.grad(o, (q1, k1, v1), g, retain_graph=True)
torch.cuda.synchronize()
print("done")
