"""Weight-gradient GEMMs of the attention block as ONE round: dW_qkv = x^T [dq|dk|dv] and
dW_o = h^T dy share the chip (both launched after the attention backward, forked on two streams)
with fewer, longer split-K slabs, against the current two sequential full-chip launches
(dW_qkv 8 slabs, dW_o 24 slabs at T = 16384).  Fewer slabs also shrink what the fused Adam reads.

    python scripts/dw_group.py            (T = 16384; T=2048 python scripts/dw_group.py)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402

dev = torch.device("cuda")
T = int(os.environ.get("T", "16384"))
ROUNDS = int(os.environ.get("ROUNDS", "7"))


def main():
    x = torch.randn(T, 640, device=dev).bfloat16()
    dq = [torch.randn(T, 512, device=dev).bfloat16() for _ in range(3)]
    h = torch.randn(T, 512, device=dev).bfloat16()
    dy = torch.randn(T, 640, device=dev).bfloat16()
    tq, Sq0, _ = hip.pick_dw_slabs(640, 3 * 512, T)
    to, So0, _ = hip.pick_dw_slabs(512, 640, T)
    print(f"T={T}: current picks dW_qkv tile {tq} S={Sq0}, dW_o tile {to} S={So0}", flush=True)
    side = torch.cuda.Stream()

    def qkv(S, tile):
        sl = torch.empty(S, 3, 640, 512, device=dev)
        return lambda: hip.gemm(x, dq[0], sl, 640, 512, T, 640, 512, 512, False, False, batch=3, sA=0,
                                sC=640 * 512, splitk=S, tile=tile, slabs=True, b_list=dq)

    def wo(S, tile):
        sl = torch.empty(S, 512, 640, device=dev)
        return lambda: hip.gemm(h, dy, sl, 512, 640, T, 512, 640, 640, False, False, sC=512 * 640, splitk=S,
                                tile=tile, slabs=True)

    def seq(a, b):
        def f():
            a()
            b()
        return f

    def conc(a, b):
        def f():
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            a()
            with torch.cuda.stream(side):
                b()
            cur.wait_stream(side)
        return f

    nkt = T // 64
    variants = {f"seq  qkv S{Sq0} + o S{So0} (current)": seq(qkv(Sq0, tq), wo(So0, to))}
    for sq, so in ((6, 6), (7, 5), (6, 8), (5, 8), (8, 8)):
        if hip.slab_count(nkt, sq) != sq or hip.slab_count(nkt, so) != so:
            continue
        variants[f"conc qkv S{sq} + o S{so}"] = conc(qkv(sq, tq), wo(so, to))
        variants[f"seq  qkv S{sq} + o S{so}"] = seq(qkv(sq, tq), wo(so, to))

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

    res = {k: [] for k in variants}
    for _ in range(ROUNDS):
        for k, f in variants.items():
            res[k].append(timeit(f))
    for k, v in res.items():
        v = sorted(v)
        print(f"{k:34s} {v[len(v) // 2]:7.2f} us (min {v[0]:.2f})", flush=True)


if __name__ == "__main__":
    main()
