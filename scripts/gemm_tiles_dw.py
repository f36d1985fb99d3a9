"""Weight-gradient slab GEMMs of the step (dW[q|k|v] = X^T dQKV, dWo = O^T dY) per LDS-DMA tile and
K-chunk count, HIP-graph timed (GEMM into slabs + the slab combine)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402
from scripts.small_kernels import graph_time  # noqa: E402

dev = torch.device("cuda")
T = 16384
for name, K, Nt, ld_b in (("dWqkv", 640, 1536, 1536), ("dWo", 512, 640, 0)):
    X = torch.randn(T, K, device=dev).bfloat16()
    dY = torch.randn(T, Nt, device=dev).bfloat16() if ld_b else torch.randn(1, Nt, device=dev).bfloat16()
    out = torch.empty(K, Nt, device=dev)
    for tile in (1282, 12883, 12884, 1284):
        for S in (4, 8, 16, 32):
            kc = T // S
            slabs = torch.empty(S, K, Nt, device=dev)

            def run():
                hip.gemm(X, dY, slabs, K, Nt, kc, K, ld_b, Nt, False, False, batch=S, sA=kc * K, sB=kc * ld_b,
                         sC=K * Nt, tile=tile)
                hip.slab_reduce(slabs, out, Nt, 0)
            us = graph_time(run)
            print(f"{name} tile={tile} S={S}: {us:7.2f} us  {2 * T * K * Nt / us / 1e6:7.1f} TF/s", flush=True)
