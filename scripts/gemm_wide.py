"""Wide-wave-tile GEMM A/B (verdict r4 item 1): the 4-wave, one-block-per-CU LDS-DMA tiles with
128-row wave tiles (codes 2522 = 256x128, 2592 = 256x192, 2552 = 256x256) against the current
tiles at the headline step's k-contiguous shapes (T = 16384), interleaved rounds in one process,
after a numerics check of every tile against the f32 torch product.

    python scripts/gemm_wide.py [case ...]     cases: qkv out dh (default: all)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402

dev = torch.device("cuda")
T = int(os.environ.get("T", "16384"))
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


def cases():
    out = {}
    x = torch.randn(T, 640, device=dev).bfloat16()
    wqkv = torch.randn(3, 512, 640, device=dev).bfloat16()
    qkv = torch.empty(T, 1536, device=dev).bfloat16()
    ref_qkv = lambda: x.float() @ wqkv.reshape(1536, 640).float().t()

    def qkv_fn(tile):
        return lambda: hip.gemm(x, wqkv, qkv, T, 512, 640, 640, 640, 1536, True, True, batch=3, sA=0, sB=512 * 640,
                                sC=512, tile=tile)
    out["qkv"] = (qkv_fn, [2561, 2562, 2522, 2592, 2552], 2 * T * 640 * 1536, qkv, ref_qkv)

    h = torch.randn(T, 512, device=dev).bfloat16()
    wo = torch.randn(640, 512, device=dev).bfloat16()
    bo = torch.randn(640, device=dev)
    y = torch.empty(T, 640, device=dev).bfloat16()
    ps = torch.empty(hip.psum_slots(T, 640) * 2, device=dev)

    def out_fn(tile):
        return lambda: hip.gemm(h, wo, y, T, 640, 512, 512, 512, 640, True, True, bias=bo, psum=ps, tile=tile)
    out["out"] = (out_fn, [1602, 2522], 2 * T * 512 * 640, y, lambda: h.float() @ wo.float().t() + bo)

    dy = torch.randn(T, 640, device=dev).bfloat16()
    won = torch.randn(512, 640, device=dev).bfloat16()
    dh = torch.empty(T, 512, device=dev).bfloat16()

    def dh_fn(tile):
        return lambda: hip.gemm(dy, won, dh, T, 512, 640, 640, 640, 512, True, True, tile=tile)
    out["dh"] = (dh_fn, [1282, 2561, 2522, 2552], 2 * T * 512 * 640, dh, lambda: dy.float() @ won.float().t())
    return out


def main():
    want = sys.argv[1:] or ["qkv", "out", "dh"]
    cs = cases()
    for name in want:
        mk, tiles, flops, outp, ref = cs[name]
        r = ref()
        fns = {}
        for t in tiles:
            outp.fill_(float("nan"))
            fns[t] = mk(t)
            fns[t]()
            torch.cuda.synchronize()
            err = ((outp.float() - r).abs().max() / r.abs().max()).item()
            ok = err < 1e-2
            print(f"{name:4s} tile {t}: max rel err {err:.2e} {'ok' if ok else 'FAIL'}", flush=True)
            if not ok:
                fns.pop(t)
        res = {t: [] for t in fns}
        for _ in range(ROUNDS):
            for t, fn in fns.items():
                res[t].append(timeit(fn))
        for t, v in res.items():
            v = sorted(v)
            med = v[len(v) // 2]
            print(f"{name:4s} tile {t}: {med:7.2f} us ({flops / med / 1e6:6.0f} TF, min {v[0]:.2f})", flush=True)


if __name__ == "__main__":
    main()
