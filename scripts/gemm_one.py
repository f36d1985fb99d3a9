"""Run ONE bench-shape GEMM configuration repeatedly (for rocprofv3 counter runs / A-B timing).

usage: python scripts/gemm_one.py {qkv,out,dattn,dwqkv,dwo,dwo_slabs} TILE [SPLITK] [ITERS]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402
from scripts.gemm_tune import timeit  # noqa: E402

dev = torch.device("cuda")
T = int(os.environ.get("T", "16384"))


def build(case, tile, sk):
    if case == "qkv":
        X, W = torch.randn(T, 640, device=dev).bfloat16(), torch.randn(1536, 640, device=dev).bfloat16()
        C = torch.empty(T, 1536, device=dev).bfloat16()
        return lambda: hip.gemm(X, W, C, T, 1536, 640, 640, 640, 1536, True, True, tile=tile), 2 * T * 1536 * 640
    if case == "out":
        X, W = torch.randn(T, 512, device=dev).bfloat16(), torch.randn(640, 512, device=dev).bfloat16()
        C = torch.empty(T, 640, device=dev).bfloat16()
        return lambda: hip.gemm(X, W, C, T, 640, 512, 512, 512, 640, True, True, tile=tile), 2 * T * 640 * 512
    if case == "dattn":
        X, W = torch.randn(T, 640, device=dev).bfloat16(), torch.randn(512, 640, device=dev).bfloat16()
        C = torch.empty(T, 512, device=dev).bfloat16()
        return lambda: hip.gemm(X, W, C, T, 512, 640, 640, 640, 512, True, True, tile=tile), 2 * T * 640 * 512
    if case == "dwqkv":
        X, dY = torch.randn(T, 640, device=dev).bfloat16(), torch.randn(T, 1536, device=dev).bfloat16()
        dW = torch.empty(3, 640, 512, device=dev)
        return (lambda: hip.gemm(X, dY, dW, 640, 512, T, 640, 1536, 512, False, False, batch=3, sA=0, sB=512,
                                 sC=640 * 512, splitk=sk, tile=tile, zero_c=True), 2 * T * 640 * 1536)
    if case == "dwo":
        X, dY = torch.randn(T, 512, device=dev).bfloat16(), torch.randn(T, 640, device=dev).bfloat16()
        dW = torch.empty(512, 640, device=dev)
        return (lambda: hip.gemm(X, dY, dW, 512, 640, T, 512, 640, 640, False, False, splitk=sk, tile=tile,
                                 zero_c=True), 2 * T * 512 * 640)
    if case == "dwo_slabs":  # split-K as a batch over K-chunks writing separate f32 slabs (no atomics)
        X, dY = torch.randn(T, 512, device=dev).bfloat16(), torch.randn(T, 640, device=dev).bfloat16()
        dW = torch.empty(sk, 512, 640, device=dev)
        kc = T // sk
        return (lambda: hip.gemm(X, dY, dW, 512, 640, kc, 512, 640, 640, False, False, batch=sk, sA=kc * 512,
                                 sB=kc * 640, sC=512 * 640, tile=tile), 2 * T * 512 * 640)
    if case == "dwall":  # the fused dWqkv as one [640][1536] GEMM (MN x MN), split-K atomics
        X, dY = torch.randn(T, 640, device=dev).bfloat16(), torch.randn(T, 1536, device=dev).bfloat16()
        dW = torch.empty(640, 1536, device=dev)
        return (lambda: hip.gemm(X, dY, dW, 640, 1536, T, 640, 1536, 1536, False, False, splitk=sk, tile=tile,
                                 zero_c=True), 2 * T * 640 * 1536)
    if case == "dwall_slabs":  # same, K-chunks as a batch writing separate f32 slabs (no atomics)
        X, dY = torch.randn(T, 640, device=dev).bfloat16(), torch.randn(T, 1536, device=dev).bfloat16()
        dW = torch.empty(sk, 640, 1536, device=dev)
        kc = T // sk
        return (lambda: hip.gemm(X, dY, dW, 640, 1536, kc, 640, 1536, 1536, False, False, batch=sk,
                                 sA=kc * 640, sB=kc * 1536, sC=640 * 1536, tile=tile), 2 * T * 640 * 1536)
    if case == "dwall_kc":  # diagnostic: operands pre-transposed to k-contiguous (ds_read_b128 path)
        Xt, dYt = torch.randn(640, T, device=dev).bfloat16(), torch.randn(1536, T, device=dev).bfloat16()
        dW = torch.empty(640, 1536, device=dev)
        return (lambda: hip.gemm(Xt, dYt, dW, 640, 1536, T, T, T, 1536, True, True, splitk=sk, tile=tile,
                                 zero_c=True), 2 * T * 640 * 1536)
    if case == "ffup":  # FF up-projection [T][640] x [640][2560], ReLU epilogue (bf16 reference for fp8)
        X, W = torch.randn(T, 640, device=dev).bfloat16(), torch.randn(2560, 640, device=dev).bfloat16()
        C = torch.empty(T, 2560, device=dev).bfloat16()
        return lambda: hip.gemm(X, W, C, T, 2560, 640, 640, 640, 2560, True, True, relu=True, tile=tile), \
            2 * T * 2560 * 640
    if case.startswith("dwslab"):  # slab-mode weight gradient: dwslab:K:N (sk = slab count)
        _, Kd, Nd = case.split(":")
        Kd, Nd = int(Kd), int(Nd)
        X, dY = torch.randn(T, Kd, device=dev).bfloat16(), torch.randn(T, Nd, device=dev).bfloat16()
        dW = torch.empty(sk, Kd, Nd, device=dev)
        return (lambda: hip.gemm(X, dY, dW, Kd, Nd, T, Kd, Nd, Nd, False, False, sC=Kd * Nd, splitk=sk, tile=tile,
                                 slabs=True), 2 * T * Kd * Nd)
    if case.startswith("dwkc"):  # diagnostic: dwkc:K:N with operands pre-transposed (ds_read_b128 path), S batch slabs
        _, Kd, Nd = case.split(":")
        Kd, Nd = int(Kd), int(Nd)
        Xt, dYt = torch.randn(Kd, T, device=dev).bfloat16(), torch.randn(Nd, T, device=dev).bfloat16()
        dW = torch.empty(sk, Kd, Nd, device=dev)
        kc = T // sk
        return (lambda: hip.gemm(Xt, dYt, dW, Kd, Nd, kc, T, T, Nd, True, True, batch=sk, sA=kc, sB=kc,
                                 sC=Kd * Nd, tile=tile), 2 * T * Kd * Nd)
    raise SystemExit(f"unknown case {case}")


def main():
    case, tile = sys.argv[1], int(sys.argv[2])
    sk = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 50
    f, flops = build(case, tile, sk)
    us = timeit(f, iters=iters, rounds=3)
    print(f"{case} tile={tile} sk={sk}: {us:.2f} us  {flops / us / 1e6:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
