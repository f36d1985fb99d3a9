"""MX-fp8 GEMM tile study: every tile of ``ljs_gemm_mx_fp8`` on the FF block's GEMM shapes and
epilogue modes, checked bit-exact against the 4-wave 128x128 kernel (tile 1282: the same MFMA
sequence per output element, so any difference is a bug) and timed with HIP events.

usage: python scripts/fp8_tiles.py [ITERS] [TILES (comma list)]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import fp8 as F  # noqa: E402

T = 16384
# (name, M, N, K, mode): the FF block at T=16384 tokens, M=640, F=2560 (case6 FF formula)
SHAPES = [
    ("up (relu, MX + MX^T)", T, 2560, 640, "qboth"),
    ("dA (fp8 mask, MX + MX^T)", T, 2560, 640, "qmask8"),
    ("down (+res)", T, 640, 2560, "res"),
    ("dX (plain)", T, 640, 2560, "plain"),
    ("dW_in f32 split 4", 640, 2560, T, "f32split"),
    ("dW_out f32 split 4", 2560, 640, T, "f32split"),
]


def setup(M, N, K, mode):
    g = torch.Generator(device="cpu").manual_seed(N * 7 + K)
    x = torch.randn(M, K, generator=g).bfloat16().cuda()
    w = torch.randn(N, K, generator=g).bfloat16().cuda()
    qa, sa = F.quant_rows(x)
    qb, sb = F.quant_rows(w)
    r = None
    if mode == "res":
        r = torch.randn(M, N, generator=g).bfloat16().cuda()
    if mode == "qmask8":
        r, _ = F.quant_rows(torch.randn(M, N, generator=g).bfloat16().cuda())
    return qa, sa, qb, sb, r


def run_one(tile, M, N, K, mode, ops):
    qa, sa, qb, sb, r = ops
    T = M
    outs = {}
    if mode in ("qboth", "qmask8"):
        outs["q"] = torch.empty(T, N, dtype=torch.uint8, device="cuda")
        outs["s"] = torch.empty(T, N // 32, dtype=torch.uint8, device="cuda")
        outs["qt"] = torch.empty(N, T, dtype=torch.uint8, device="cuda")
        outs["st"] = torch.empty(N, T // 32, dtype=torch.uint8, device="cuda")
        c = None
    elif mode == "f32split":
        c = torch.empty(4, T, N, dtype=torch.float32, device="cuda")
        outs["c"] = c
    else:
        c = torch.empty(T, N, dtype=torch.bfloat16, device="cuda")
        outs["c"] = c

    def go():
        if mode == "qboth":
            F.gemm_mx(qa, sa, qb, sb, T, N, K, None, relu=True, qout=(outs["q"], outs["s"]),
                      qtout=(outs["qt"], outs["st"]), tile=tile)
        elif mode == "qmask8":
            F.gemm_mx(qa, sa, qb, sb, T, N, K, None, res=r, res_mode="mask", qout=(outs["q"], outs["s"]),
                      qtout=(outs["qt"], outs["st"]), tile=tile)
        elif mode == "res":
            F.gemm_mx(qa, sa, qb, sb, T, N, K, c, res=r, tile=tile)
        elif mode == "f32split":
            F.gemm_mx(qa, sa, qb, sb, T, N, K, c, nsplit=4, tile=tile)
        else:
            F.gemm_mx(qa, sa, qb, sb, T, N, K, c, tile=tile)
    return go, outs


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    tiles = [int(t) for t in sys.argv[2].split(",")] if len(sys.argv) > 2 else \
        [1282, 256256, 256128, 256160, 128320, 128256, 128128, 128160, 3128128, 3128160, 3128256, 3256128]
    bad = 0
    for name, M, N, K, mode in SHAPES:
        ops = setup(M, N, K, mode)
        ref = None
        for tile in tiles:
            go, outs = run_one(tile, M, N, K, mode, ops)
            try:
                go()
                torch.cuda.synchronize()
            except RuntimeError as e:
                print(f"{name:28s} tile {tile}: rejected ({e})", flush=True)
                continue
            if ref is None:
                ref = {k: v.clone() for k, v in outs.items()}
                same = "ref"
            else:
                same = "bit-exact" if all(torch.equal(ref[k], outs[k]) for k in ref) else "MISMATCH"
                if same == "MISMATCH":
                    bad += 1
                    for k in ref:
                        d = (ref[k].float() - outs[k].float()).abs()
                        print(f"    {k}: {int((d > 0).sum())} of {d.numel()} differ, max {float(d.max()):.3g}",
                              flush=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(3):
                go()
            e0.record()
            for _ in range(iters):
                go()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / iters * 1e3
            flops = 2.0 * M * N * K
            print(f"{name:28s} tile {tile:7d}: {us:7.1f} us  {flops / us / 1e6:6.0f} TF  {same}", flush=True)
    print("mismatches:", bad, flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
