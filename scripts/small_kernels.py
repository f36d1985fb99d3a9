"""Time the bench step's memory-bound kernels in isolation, each replayed from a HIP graph of 20
launches (so host launch cost is excluded), at the bench shapes (T = 16384 tokens).

usage: python scripts/small_kernels.py [names...]   (LJS_SUM_BLOCKS=N to override sum_all's grid cap)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402

dev = torch.device("cuda")
T = 16384


def graph_time(fn, n=20, reps=5):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        res.append(a.elapsed_time(b) * 1e3 / n)
    res.sort()
    return res[len(res) // 2]


def main():
    which = sys.argv[1:] or ["sum", "cast", "slab_qkv", "slab_o", "adam"]
    out = {}
    y = torch.randn(T, 640, device=dev).bfloat16()
    x = torch.randn(T, 640, device=dev)
    xb = torch.empty(T, 640, device=dev, dtype=torch.bfloat16)
    if "sum" in which:
        out["sum_all bf16 [T,640]"] = graph_time(lambda: hip._sum_all_raw(y, torch.bfloat16))
    if "cast" in which:
        out["cast f32->bf16 [T,640]"] = graph_time(lambda: hip._cast_raw(x, torch.bfloat16))
    if "slab_qkv" in which:
        sl = torch.randn(8, 640, 1536, device=dev)
        o = torch.empty(3, 640, 512, device=dev)
        out["slab_reduce 8x[640,1536]"] = graph_time(lambda: hip.slab_reduce(sl, o, 512, 640 * 512))
    if "slab_o" in which:
        sl = torch.randn(16, 512, 640, device=dev)
        o = torch.empty(512, 640, device=dev)
        out["slab_reduce 16x[512,640]"] = graph_time(lambda: hip.slab_reduce(sl, o, 640, 0))
    if "adam" in which:
        ps = [torch.randn(640, 512, device=dev) for _ in range(3)] + [torch.randn(512, 640, device=dev),
                                                                     torch.randn(640, device=dev)]
        gs = [torch.randn_like(p) for p in ps]
        ms = [torch.zeros_like(p) for p in ps]
        vs = [torch.zeros_like(p) for p in ps]
        step = torch.zeros((), dtype=torch.int32, device=dev)
        ents = list(zip(ps, gs, ms, vs))
        out["adam_multi 5 params"] = graph_time(lambda: hip.adam_multi(ents, step, 1e-3, 0.9, 0.999, 1e-8, 0.0))
    for k, v in out.items():
        print(f"{k:32s} {v:8.2f} us", flush=True)


if __name__ == "__main__":
    main()
