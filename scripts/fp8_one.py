"""Run ONE MX-fp8 GEMM configuration repeatedly (rocprofv3 counter runs): T x N x K, tile.

usage: python scripts/fp8_one.py N K TILE [ITERS] [qout|qmask|res|qonly|qboth]  (prints the mean time)

qboth: the FF up projection of the fused MX-fp8 block (ReLU, MX copy along N AND the transposed
MX copy along tokens, no bf16 output).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import fp8 as F  # noqa: E402

T = 16384


def main():
    N, K, tile = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    mode = sys.argv[5] if len(sys.argv) > 5 else ""
    qo = mode in ("qout", "qmask", "qonly", "qboth")
    qt = torch.empty(N, T, dtype=torch.uint8, device="cuda") if mode == "qboth" else None
    st = torch.empty(N, T // 32, dtype=torch.uint8, device="cuda") if mode == "qboth" else None
    r = torch.randn(T, N, device="cuda").bfloat16() if mode in ("qmask", "res") else None
    x = torch.randn(T, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    qa, sa = F.quant_rows(x)
    qb, sb = F.quant_rows(w)
    c = torch.empty(T, N, device="cuda").bfloat16()
    q = torch.empty(T, N, dtype=torch.uint8, device="cuda")
    s = torch.empty(T, N // 32, dtype=torch.uint8, device="cuda")
    def run():
        F.gemm_mx(qa, sa, qb, sb, T, N, K, None if mode in ("qonly", "qboth") else c, qout=(q, s) if qo else None,
                  tile=tile, res=r, res_mode="mask" if mode == "qmask" else "add",
                  relu=mode in ("qout", "relu", "qonly", "qboth"), qtout=(qt, st) if qt is not None else None)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    print(f"N={N} K={K} tile={tile} mode={mode or 'plain'}: {e0.elapsed_time(e1) / iters * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
