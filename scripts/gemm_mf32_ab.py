"""32x32x16 vs 16x16x32 MFMA lean K-loop GEMMs at the step's k-contiguous shapes (verdict r5 item
2a): correctness against an fp32 reference, then interleaved timing rounds in one process.
Tile code + 100000 forces the 16x16x32 lean kernel, + 300000 the 32x32x16 one.

    python scripts/gemm_mf32_ab.py            (T = 16384 and T = 2048 cases)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402

dev = torch.device("cuda")
ROUNDS = int(os.environ.get("ROUNDS", "7"))


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
    g = torch.Generator(device=dev).manual_seed(T)
    x = torch.randn(T, 640, device=dev, generator=g).bfloat16()
    wqkv = (torch.randn(3, 512, 640, device=dev, generator=g) * 0.05).bfloat16()
    qkv = torch.empty(T, 1536, device=dev).bfloat16()
    ref_qkv = x.float() @ wqkv.float().reshape(1536, 640).t()

    def qkv_fn(tile):
        return lambda: hip.gemm(x, wqkv, qkv, T, 512, 640, 640, 640, 1536, True, True, batch=3, sA=0, sB=512 * 640,
                                sC=512, tile=tile)
    h = torch.randn(T, 512, device=dev, generator=g).bfloat16()
    wo = (torch.randn(640, 512, device=dev, generator=g) * 0.05).bfloat16()
    bo = torch.randn(640, device=dev, generator=g)
    y = torch.empty(T, 640, device=dev).bfloat16()
    ps = torch.zeros(hip.psum_slots(T, 640) * 2, device=dev)
    ref_y = h.float() @ wo.float().t() + bo

    def out_fn(tile):
        return lambda: hip.gemm(h, wo, y, T, 640, 512, 512, 512, 640, True, True, bias=bo, psum=ps, tile=tile)
    dy = torch.randn(T, 640, device=dev, generator=g).bfloat16()
    won = (torch.randn(512, 640, device=dev, generator=g) * 0.05).bfloat16()
    dh = torch.empty(T, 512, device=dev).bfloat16()
    ref_dh = dy.float() @ won.float().t()

    def dh_fn(tile):
        return lambda: hip.gemm(dy, won, dh, T, 512, 640, 640, 640, 512, True, True, tile=tile)
    if T >= 8192:
        out += [("qkv 2562", qkv_fn, 2562, qkv, ref_qkv), ("qkv 2561", qkv_fn, 2561, qkv, ref_qkv),
                ("out 1602", out_fn, 1602, y, ref_y), ("dh 1282", dh_fn, 1282, dh, ref_dh)]
    else:
        out += [("qkv 12883", qkv_fn, 12883, qkv, ref_qkv), ("dh 1282", dh_fn, 1282, dh, ref_dh)]
    return out


def main():
    for T in (16384, 2048):
        for name, mk, tile, outbuf, ref in cases(T):
            errs = {}
            for base in (100000, 300000):
                outbuf.fill_(float("nan"))
                mk(base + tile)()
                torch.cuda.synchronize()
                errs[base] = ((outbuf.float() - ref).abs().max() / ref.abs().max()).item()
            ts = {100000: [], 300000: []}
            for _ in range(ROUNDS):
                for base in (100000, 300000):
                    ts[base].append(timeit(mk(base + tile)))
            med = {b: sorted(v)[len(v) // 2] for b, v in ts.items()}
            print(f"T={T:6d} {name:10s} 16x16x32 {med[100000]:7.2f} us (err {errs[100000]:.2e})   "
                  f"32x32x16 {med[300000]:7.2f} us (err {errs[300000]:.2e})   "
                  f"ratio {med[300000] / med[100000]:.3f}   all: {[round(v, 1) for v in ts[300000]]}", flush=True)


if __name__ == "__main__":
    main()
