"""MX-fp8 vs bf16 GEMM times at the FF-layer shapes (T=16384 tokens, M=640, ff=2560), HIP-graph
replays of 10 launches; plus the quantization passes the fp8 path needs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import fp8 as F  # noqa: E402
from learning_jax_sharding_amd.ops import hip  # noqa: E402
from scripts.gemm_small import graph_time  # noqa: E402

dev = torch.device("cuda")
T = int(os.environ.get("T", "16384"))


def main():
    for name, K, N in (("ff_up", 640, 2560), ("ff_down", 2560, 640), ("dX_ffdown", 640, 2560), ("dX_ffup", 2560, 640)):
        x = torch.randn(T, K, device=dev).bfloat16()
        w = torch.randn(N, K, device=dev).bfloat16()   # k-contiguous B
        c = torch.empty(T, N, device=dev).bfloat16()
        fl = 2 * T * K * N
        for tile in ((2561, 1602, 1282) if N % 160 == 0 else (2561, 1282)):
            us = graph_time(lambda: hip.gemm(x, w, c, T, N, K, K, K, N, True, True, tile=tile), reps=10)
            print(f"{name} bf16 tile={tile}: {us:.1f} us {fl / us / 1e6:.0f} TF", flush=True)
        qa, sa = F.quant_rows(x)
        qb, sb = F.quant_rows(w)
        for tile in (1282, 1283, 2562, 2563):
            us = graph_time(lambda: F.gemm_mx(qa, sa, qb, sb, T, N, K, c, tile=tile), reps=10)
            print(f"{name} fp8 tile={tile}: {us:.1f} us {fl / us / 1e6:.0f} TF", flush=True)
        q = torch.empty(T, N, dtype=torch.uint8, device=dev)
        s = torch.empty(T, N // 32, dtype=torch.uint8, device=dev)
        us = graph_time(lambda: F.gemm_mx(qa, sa, qb, sb, T, N, K, c, qout=(q, s)), reps=10)
        print(f"{name} fp8 auto + quantized output copy: {us:.1f} us", flush=True)
        us = graph_time(lambda: F.quant_rows(x), reps=10)
        print(f"{name} quant_rows of the [{T}, {K}] input: {us:.1f} us", flush=True)


if __name__ == "__main__":
    main()
