"""Time the attention kernels in isolation at the bench shape (B=64, S=256, H=8, D=64)."""
import json
import sys

import torch

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402
from scripts.gemm_tune import timeit  # noqa: E402

dev = torch.device("cuda")
B, S, H, D = (int(a) for a in (sys.argv[1:5] if len(sys.argv) > 4 else (64, 256, 8, 64)))
qkv = torch.randn(B, S, 3, H, D, device=dev).bfloat16()
q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
scale = D ** -0.5
res = {}
res["fwd"] = timeit(lambda: hip.attention(q, k, v, scale))
q1, k1, v1 = (t.detach().requires_grad_() for t in (q, k, v))
o = hip.attention(q1, k1, v1, scale)
g = torch.randn_like(o)
res["fwd+bwd"] = timeit(lambda: torch.autograd.grad(hip.attention(q1, k1, v1, scale), (q1, k1, v1), g))
hip.set_attention_bwd_fused(False)
res["fwd+bwd split"] = timeit(lambda: torch.autograd.grad(hip.attention(q1, k1, v1, scale), (q1, k1, v1), g))
hip.set_attention_bwd_fused(None)
# torch SDPA (ROCm flash / efficient backends) on the same problem, (B, H, S, D) layout
import torch.nn.functional as F
qt, kt, vt = (t.transpose(1, 2).contiguous() for t in (q, k, v))
try:
    res["torch sdpa fwd"] = timeit(lambda: F.scaled_dot_product_attention(qt, kt, vt, scale=scale))
    qt1, kt1, vt1 = (t.detach().requires_grad_() for t in (qt, kt, vt))
    ot = F.scaled_dot_product_attention(qt1, kt1, vt1, scale=scale)
    gt = torch.randn_like(ot)
    res["torch sdpa fwd+bwd"] = timeit(lambda: torch.autograd.grad(
        F.scaled_dot_product_attention(qt1, kt1, vt1, scale=scale), (qt1, kt1, vt1), gt))
except Exception as e:  # noqa: BLE001
    print("sdpa failed:", e)
fl = 4 * B * H * S * S * D
res["fwd TFLOPS"] = fl / res["fwd"] / 1e6
res["fwd+bwd TFLOPS"] = 3.5 * fl / res["fwd+bwd"] / 1e6
for kk, vv in res.items():
    print(f"{kk:20s} {vv:10.2f}")
json.dump(res, open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "attn_bench.json"), "w"))
