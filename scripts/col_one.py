"""Cast-on-load QKV GEMM variants at T tokens (A/B of the f32-A LDS-DMA kernel)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402
from scripts.gemm_tune import timeit  # noqa: E402

T = int(os.environ.get("T", "16384"))
dev = torch.device("cuda")
x = torch.randn(T, 640, device=dev)
xb = x.bfloat16()
w = torch.randn(3, 512, 640, device=dev).bfloat16()
out = torch.empty(T, 1536, device=dev).bfloat16()
cp = torch.empty(T, 640, device=dev).bfloat16()
cases = {
    "cast+2561": lambda: (hip._cast_raw(x, torch.bfloat16), hip.gemm(xb, w, out, T, 512, 640, 640, 640, 1536, True, True,
                                                                    batch=3, sB=512 * 640, sC=512, tile=2561)),
    "cast+1282": lambda: (hip._cast_raw(x, torch.bfloat16), hip.gemm(xb, w, out, T, 512, 640, 640, 640, 1536, True, True,
                                                                    batch=3, sB=512 * 640, sC=512, tile=1282)),
    "bf16 12883": lambda: hip.gemm(xb, w, out, T, 512, 640, 640, 640, 1536, True, True, batch=3, sB=512 * 640, sC=512,
                                   tile=12883),
    "f32A+copy": lambda: hip.gemm(x, w, out, T, 512, 640, 640, 640, 1536, True, True, batch=3, sB=512 * 640, sC=512,
                                  acopy=cp),
    "f32A nocopy": lambda: hip.gemm(x, w, out, T, 512, 640, 640, 640, 1536, True, True, batch=3, sB=512 * 640, sC=512),
}
for k, f in cases.items():
    print(f"T={T} {k}: {timeit(f, iters=50, rounds=3):.2f} us", flush=True)
