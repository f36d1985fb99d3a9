"""Time GEMM configurations on the MI355X (interleaved rounds in one process)."""
import itertools
import json
import sys

import torch

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402

dev = torch.device("cuda")


def timeit(fn, iters=20, rounds=5):
    best = []
    for _ in range(rounds):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        best.append(s.elapsed_time(e) / iters * 1e3)
    best.sort()
    return best[len(best) // 2]


def main():
    T = 16384
    res = {}
    X = torch.randn(T, 640, device=dev).bfloat16()
    dQKV = torch.randn(T, 1536, device=dev).bfloat16()
    O = torch.randn(T, 512, device=dev).bfloat16()
    dY = torch.randn(T, 640, device=dev).bfloat16()
    # dW_qkv = X^T dQKV (batched 3 x [640][512]); dWo = O^T dY ([512][640])
    for tile, sk in itertools.product([64, 128], [1, 2, 3, 4, 6, 8]):
        dW = torch.empty(3, 640, 512, device=dev)
        f = lambda: hip.gemm(X, dQKV, dW, 640, 512, T, 640, 1536, 512, False, False, batch=3, sA=0, sB=512,
                             sC=640 * 512, splitk=sk, tile=tile, zero_c=sk > 1)
        us = timeit(f)
        res[f"dWqkv tile{tile} sk{sk}"] = us
        dWo = torch.empty(512, 640, device=dev)
        g = lambda: hip.gemm(O, dY, dWo, 512, 640, T, 512, 640, 640, False, False, splitk=sk, tile=tile,
                             zero_c=sk > 1)
        res[f"dWo tile{tile} sk{sk}"] = timeit(g)
    # forward GEMMs
    Wt = torch.randn(3, 512, 640, device=dev).bfloat16()
    out = torch.empty(T, 1536, device=dev).bfloat16()
    for tile in (64, 128):
        f = lambda: hip.gemm(X, Wt, out, T, 512, 640, 640, 640, 1536, True, True, batch=3, sA=0, sB=512 * 640,
                             sC=512, tile=tile)
        res[f"qkv fwd tile{tile}"] = timeit(f)
        Wo = torch.randn(640, 512, device=dev).bfloat16()
        y = torch.empty(T, 640, device=dev).bfloat16()
        g = lambda: hip.gemm(O, Wo, y, T, 640, 512, 512, 512, 640, True, True, tile=tile)
        res[f"out fwd tile{tile}"] = timeit(g)
    # square reference point
    A = torch.randn(8192, 8192, device=dev).bfloat16()
    Bt = torch.randn(8192, 8192, device=dev).bfloat16()
    C = torch.empty(8192, 8192, device=dev).bfloat16()
    us = timeit(lambda: hip.gemm(A, Bt, C, 8192, 8192, 8192, 8192, 8192, 8192, True, True, tile=128), iters=5)
    res["8192^3 NT tile128 (TFLOPS)"] = 2 * 8192 ** 3 / us / 1e6
    us = timeit(lambda: torch.matmul(A, Bt.t()), iters=5)
    res["8192^3 torch/hipBLASLt (TFLOPS)"] = 2 * 8192 ** 3 / us / 1e6
    for k, v in res.items():
        print(f"{k:40s} {v:10.2f}")
    json.dump(res, open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "gemm_tune.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
