"""Where does a bench-shape GEMM spend its time?  K-scaling + output-dtype probes.

For the forward projection shape (M = 16384 tokens, N = 1536, K = 640) time the kernel at
K = 640 .. 10240: the slope is the per-K-tile cost, the intercept the fixed (prologue +
epilogue + launch) cost.  Usage: ``python scripts/gemm_probe.py``.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402
from scripts.gemm_tune import timeit  # noqa: E402

dev = torch.device("cuda")


def main():
    T = 16384
    print(f"{'case':44s} {'us':>9s} {'TF/s':>8s}")
    tiles = (128, 2561, 1284, 1282)
    for N in (1536, 640, 512):
        for K in (640, 2560):
            X = torch.randn(T, K, device=dev).bfloat16()
            W = torch.randn(N, K, device=dev).bfloat16()
            for out_dt in (torch.bfloat16, torch.float32):
                C = torch.empty(T, N, device=dev, dtype=out_dt)
                for tile in tiles:
                    f = lambda: hip.gemm(X, W, C, T, N, K, K, K, N, True, True, tile=tile)  # noqa: E731
                    us = timeit(f)
                    print(f"M={T} N={N} K={K} out={str(out_dt)[6:]} tile={tile}".ljust(44),
                          f"{us:9.2f} {2 * T * N * K / us / 1e6:8.1f}", flush=True)
    # weight-grad shapes: dW[M][N] = X^T dY, both operands m/n-contiguous, split-K atomics
    for (M, N, nb) in ((640, 512, 3), (512, 640, 1)):
        X = torch.randn(T, M, device=dev).bfloat16()
        dY = torch.randn(T, nb * N, device=dev).bfloat16()
        dW = torch.empty(nb, M, N, device=dev)
        for tile in tiles:
            for sk in (2, 4, 6, 8, 12, 16):
                f = lambda: hip.gemm(X, dY, dW, M, N, T, M, nb * N, N, False, False, batch=nb, sA=0, sB=N,  # noqa
                                     sC=M * N, splitk=sk, tile=tile, zero_c=True)
                us = timeit(f)
                print(f"dW M={M} N={N}x{nb} K={T} tile={tile} sk={sk}".ljust(44),
                      f"{us:9.2f} {2 * T * M * N * nb / us / 1e6:8.1f}", flush=True)
    for n in (4096, 8192):
        A = torch.randn(n, n, device=dev).bfloat16()
        Bt = torch.randn(n, n, device=dev).bfloat16()
        C = torch.empty(n, n, device=dev).bfloat16()
        for tile in tiles:
            us = timeit(lambda: hip.gemm(A, Bt, C, n, n, n, n, n, n, True, True, tile=tile), iters=5)
            print(f"{n}^3 NT tile{tile}".ljust(44), f"{us:9.2f} {2 * n ** 3 / us / 1e6:8.1f}")
        us = timeit(lambda: torch.matmul(A, Bt.t()), iters=5)
        print(f"{n}^3 hipBLASLt".ljust(44), f"{us:9.2f} {2 * n ** 3 / us / 1e6:8.1f}")


if __name__ == "__main__":
    main()
