"""hipBLASLt (torch.matmul) vs the hand-written kernel on the attention block's GEMM shapes."""
import json
import sys

import torch

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.gemm_tune import timeit  # noqa: E402

dev = torch.device("cuda")
T = 16384
X = torch.randn(T, 640, device=dev).bfloat16()
dQKV = torch.randn(T, 1536, device=dev).bfloat16()
O = torch.randn(T, 512, device=dev).bfloat16()
dY = torch.randn(T, 640, device=dev).bfloat16()
Wqkv = torch.randn(640, 1536, device=dev).bfloat16()
Wo = torch.randn(512, 640, device=dev).bfloat16()
bo = torch.randn(640, device=dev).bfloat16()
res = {}
res["blas dWqkv X^T dQKV (f32 out)"] = timeit(lambda: torch.matmul(X.t(), dQKV, out_dtype=torch.float32)
                                             if hasattr(torch, "_foo") else torch.mm(X.t(), dQKV).float())
res["blas dWqkv X^T dQKV (bf16 out)"] = timeit(lambda: torch.mm(X.t(), dQKV))
res["blas dWo O^T dY (bf16 out)"] = timeit(lambda: torch.mm(O.t(), dY))
res["blas qkv fwd X Wqkv"] = timeit(lambda: torch.mm(X, Wqkv))
res["blas out fwd addmm"] = timeit(lambda: torch.addmm(bo, O, Wo))
res["blas dO = dY Wo^T"] = timeit(lambda: torch.mm(dY, Wo.t()))
for k, v in res.items():
    print(f"{k:40s} {v:10.2f} us")
json.dump(res, open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "blas_compare.json"), "w"), indent=1)
