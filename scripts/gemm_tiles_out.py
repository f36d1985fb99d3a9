"""The step's k-contiguous GEMM shapes (T = 16384 rows, +bias) on each LDS-DMA tile, HIP-graph timed."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402
from scripts.small_kernels import graph_time  # noqa: E402

dev = torch.device("cuda")
T = 16384
for (N, K) in ((640, 512), (640, 2560), (1536, 640), (512, 640), (2560, 640)):
    X = torch.randn(T, K, device=dev).bfloat16()
    W = torch.randn(N, K, device=dev).bfloat16()
    b = torch.randn(N, device=dev)
    C = torch.empty(T, N, device=dev).bfloat16()
    for tile in (1282, 1602, 2561):
        if tile == 1602 and N % 160:
            continue
        us = graph_time(lambda: hip.gemm(X, W, C, T, N, K, K, K, N, True, True, bias=b, tile=tile))
        print(f"N={N} K={K} tile={tile}: {us:7.2f} us  {2 * T * N * K / us / 1e6:7.1f} TF/s", flush=True)
