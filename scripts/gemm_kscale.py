"""Fixed vs per-K-tile cost of the LDS-DMA GEMMs: time C[T,N] = X[T,K] W[N,K]^T at K = 640..2560
(t(K) = a + b K: a = prologue/epilogue/launch cost per block round, b = K-loop cost)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402
from scripts.small_kernels import graph_time  # noqa: E402

dev = torch.device("cuda")
T = 16384
for N, tile in ((1536, 2561), (640, 1282), (1536, 1282)):
    for K in (640, 1280, 2560):
        X = torch.randn(T, K, device=dev).bfloat16()
        W = torch.randn(N, K, device=dev).bfloat16()
        C = torch.empty(T, N, device=dev).bfloat16()
        us = graph_time(lambda: hip.gemm(X, W, C, T, N, K, K, K, N, True, True, tile=tile))
        print(f"N={N} tile={tile} K={K}: {us:8.2f} us  {2 * T * N * K / us / 1e6:7.1f} TF/s", flush=True)
