"""Lean K-loop GEMM (gemm.hip gemm_lean_kernel) against the general LDS-DMA kernel at the step's
k-contiguous shapes: outputs must be bit-identical, then interleaved timing rounds in one process.
Tile code + 100000 forces the lean kernel, + 200000 the general one.

    python scripts/gemm_lean_ab.py            (T = 16384 and T = 2048 cases)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402

dev = torch.device("cuda")
ROUNDS = int(os.environ.get("ROUNDS", "7"))
LEAN = 100000


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def cases(T):
    out = []
    x = torch.randn(T, 640, device=dev).bfloat16()
    wqkv = torch.randn(3, 512, 640, device=dev).bfloat16()
    qkv = torch.empty(T, 1536, device=dev).bfloat16()

    def qkv_fn(tile):
        return lambda: hip.gemm(x, wqkv, qkv, T, 512, 640, 640, 640, 1536, True, True, batch=3, sA=0, sB=512 * 640,
                                sC=512, tile=tile)
    h = torch.randn(T, 512, device=dev).bfloat16()
    wo = torch.randn(640, 512, device=dev).bfloat16()
    bo = torch.randn(640, device=dev)
    y = torch.empty(T, 640, device=dev).bfloat16()
    ps = torch.empty(hip.psum_slots(T, 640) * 2, device=dev)

    def out_fn(tile):
        return lambda: hip.gemm(h, wo, y, T, 640, 512, 512, 512, 640, True, True, bias=bo, psum=ps, tile=tile)
    dy = torch.randn(T, 640, device=dev).bfloat16()
    won = torch.randn(512, 640, device=dev).bfloat16()
    dh = torch.empty(T, 512, device=dev).bfloat16()
    r = torch.randn(T, 512, device=dev).bfloat16()

    def dh_fn(tile):
        return lambda: hip.gemm(dy, won, dh, T, 512, 640, 640, 640, 512, True, True, tile=tile)

    def dhm_fn(tile):   # ReLU-mask epilogue operand (RES 1)
        return lambda: hip.gemm(dy, won, dh, T, 512, 640, 640, 640, 512, True, True, tile=tile, res=r, res_ld=512,
                                res_mode="mask")
    big = T >= 8192
    out.append(("qkv", qkv_fn, [2561, 2562] if big else [12883], 2 * T * 640 * 1536, qkv))
    out.append(("out", out_fn, [1602] if big else [644], 2 * T * 512 * 640, y))
    out.append(("dh", dh_fn, [1282, 2561] if big else [644, 12883], 2 * T * 512 * 640, dh))
    out.append(("dh+mask", dhm_fn, [1282] if big else [12883], 2 * T * 512 * 640, dh))
    return out


def main():
    for T in (16384, 2048):
        for name, mk, tiles, flops, outp in cases(T):
            fns = {}
            for t in tiles:
                outp.zero_()
                mk(t + 2 * LEAN)()
                torch.cuda.synchronize()
                ref = outp.clone()
                outp.fill_(float("nan"))
                mk(t + LEAN)()
                torch.cuda.synchronize()
                iv = torch.int16
                same = torch.equal(outp.view(iv), ref.view(iv))
                print(f"T={T} {name:8s} tile {t}: lean bit-exact {'ok' if same else 'FAIL'}", flush=True)
                if not same:
                    bad = (outp.view(iv) != ref.view(iv)).nonzero()
                    print("   first mismatches", bad[:5].tolist(), flush=True)
                    continue
                fns[t + 2 * LEAN] = mk(t + 2 * LEAN)
                fns[t + LEAN] = mk(t + LEAN)
            res = {t: [] for t in fns}
            for _ in range(ROUNDS):
                for t, fn in fns.items():
                    res[t].append(timeit(fn))
            for t, v in res.items():
                v = sorted(v)
                med = v[len(v) // 2]
                kind = "general" if t >= 2 * LEAN else "lean"
                print(f"T={T} {name:8s} tile {t % LEAN} {kind:7s}: {med:7.2f} us ({flops / med / 1e6:6.0f} TF, "
                      f"min {v[0]:.2f})", flush=True)


if __name__ == "__main__":
    main()
