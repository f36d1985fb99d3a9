"""Tile sweep for the GEMMs of the reference-shape step (B=8 x 256 = 2048 tokens, M=640,
inner 512): forward QKV / out-projection, dX of the out-projection, and the weight-gradient
slab GEMMs (K-chunks as a batch into f32 slabs).  Times are medians of HIP-graph replays of 20
launches (launch gaps included, as in the captured step)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402

dev = torch.device("cuda")
T = int(os.environ.get("T", "2048"))


def graph_time(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    ts.sort()
    return ts[2]


def main():
    X = torch.randn(T, 640, device=dev).bfloat16()
    H = torch.randn(T, 512, device=dev).bfloat16()
    Wqkv = torch.randn(1536, 640, device=dev).bfloat16()
    Wo_t = torch.randn(640, 512, device=dev).bfloat16()
    Wo = torch.randn(512, 640, device=dev).bfloat16()
    dY = torch.randn(T, 640, device=dev).bfloat16()
    dQKV = torch.randn(T, 1536, device=dev).bfloat16()
    C1 = torch.empty(T, 1536, device=dev).bfloat16()
    C2 = torch.empty(T, 640, device=dev).bfloat16()
    C3 = torch.empty(T, 512, device=dev).bfloat16()
    W3 = Wqkv.view(3, 512, 640)
    fw = {
        "qkv": (lambda t: hip.gemm(X, Wqkv, C1, T, 1536, 640, 640, 640, 1536, True, True, tile=t), 2 * T * 1536 * 640),
        "qkv3": (lambda t: hip.gemm(X, W3, C1, T, 512, 640, 640, 640, 1536, True, True, batch=3, sB=512 * 640, sC=512,
                                    tile=t), 2 * T * 1536 * 640),
        "out": (lambda t: hip.gemm(H, Wo_t, C2, T, 640, 512, 512, 512, 640, True, True, tile=t), 2 * T * 640 * 512),
        "dh": (lambda t: hip.gemm(dY, Wo, C3, T, 512, 640, 640, 640, 512, True, True, tile=t), 2 * T * 640 * 512),
    }
    for name, (mk, fl) in fw.items():
        for t in (64, 128, 643, 644, 1282, 1284, 12883, 12884, 2561, 1602):
            us = graph_time(lambda: mk(t))
            print(f"{name} tile={t}: {us:.2f} us {fl / us / 1e6:.0f} TF", flush=True)
    if os.environ.get("FWD_ONLY") == "1":
        return
    # weight gradients: S K-chunks into f32 slabs (+ the combine), tile choices
    for name, A, B, K_, N_ in (("dwo", H, dY, 512, 640), ("dwqkv", X, dQKV, 640, 1536)):
        out = torch.empty(K_, N_, device=dev)
        for t in (643, 644, 1282):
            for S in (1, 2, 4, 8, 16):
                if T % (64 * S):
                    continue
                kc = T // S
                slabs = torch.empty((S, K_, N_), device=dev)

                def run(t=t, S=S, kc=kc, slabs=slabs):
                    hip.gemm(A, B, slabs, K_, N_, kc, K_, N_, N_, False, False, batch=S, sA=kc * K_, sB=kc * N_,
                             sC=K_ * N_, tile=t)
                    if S > 1:
                        hip.slab_reduce(slabs, out, N_, 0)
                us = graph_time(run)
                print(f"{name} tile={t} S={S}: {us:.2f} us {2 * T * K_ * N_ / us / 1e6:.0f} TF", flush=True)


if __name__ == "__main__":
    main()
