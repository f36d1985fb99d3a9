"""Where the MX-fp8 up projection's time goes (verdict r5 item 5): the T=16384 x 2560 x 640 GEMM
timed with its full epilogue (ReLU + row-blocked MX copy + transposed MX copy: the FF block's
fixed-flag kernel) and with parts of that epilogue removed, plus the K-loop alone (f32 output of
one split, no MX work), on the 4-wave 128x128 kernel and the other tiles.

    python scripts/fp8_upproj_probe.py [ITERS]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import fp8 as F  # noqa: E402

T, N, K = 16384, 2560, 640


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.randn(T, K, generator=g).bfloat16().cuda()
    w = torch.randn(N, K, generator=g).bfloat16().cuda()
    qa, sa = F.quant_rows(x)
    qb, sb = F.quant_rows(w)
    q = torch.empty(T, N, dtype=torch.uint8, device="cuda")
    s = torch.empty(T, N // 32, dtype=torch.uint8, device="cuda")
    qt = torch.empty(N, T, dtype=torch.uint8, device="cuda")
    st = torch.empty(N, T // 32, dtype=torch.uint8, device="cuda")
    cb = torch.empty(T, N, dtype=torch.bfloat16, device="cuda")
    cf = torch.empty(T, N, dtype=torch.float32, device="cuda")
    cases = [
        ("relu + MX + MX^T (block's kernel)", 1282, dict(out=None, relu=True, qout=(q, s), qtout=(qt, st))),
        ("relu + MX + MX^T, 3 stages", 1283, dict(out=None, relu=True, qout=(q, s), qtout=(qt, st))),
        ("relu + MX + MX^T, 256x128 8w", 2562, dict(out=None, relu=True, qout=(q, s), qtout=(qt, st))),
        ("relu + MX + MX^T, 8w 256x256", 256256, dict(out=None, relu=True, qout=(q, s), qtout=(qt, st))),
        ("relu + MX + MX^T, 8w 256x160", 256160, dict(out=None, relu=True, qout=(q, s), qtout=(qt, st))),
        ("relu + MX + MX^T, 8w 128x256", 128256, dict(out=None, relu=True, qout=(q, s), qtout=(qt, st))),
        ("relu + MX only", 1282, dict(out=None, relu=True, qout=(q, s))),
        ("relu + MX^T + bf16", 1282, dict(out=cb, relu=True, qtout=(qt, st))),
        ("relu, bf16 out", 1282, dict(out=cb, relu=True)),
        ("f32 out (K-loop + plain stores)", 1282, dict(out=cf)),
        ("f32 out, 3 stages", 1283, dict(out=cf)),
    ]
    flops = 2.0 * T * N * K
    for name, tile, kw in cases:
        def go():
            F.gemm_mx(qa, sa, qb, sb, T, N, K, kw["out"], relu=kw.get("relu", False), qout=kw.get("qout"),
                      qtout=kw.get("qtout"), tile=tile)
        try:
            go()
            torch.cuda.synchronize()
        except (RuntimeError, AssertionError) as e:
            print(f"{name:36s} tile {tile:7d}: rejected ({e})", flush=True)
            continue
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                go()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / iters * 1e3)
        ts.sort()
        us = ts[len(ts) // 2]
        print(f"{name:36s} tile {tile:7d}: {us:7.1f} us  {flops / us / 1e6:6.0f} TF  (all {[round(t, 1) for t in ts]})",
              flush=True)


if __name__ == "__main__":
    main()
