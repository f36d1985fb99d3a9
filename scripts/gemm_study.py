"""Every bench-shape GEMM of the case6 train step under every kernel/tile choice, plus the
hipBLASLt (torch.mm) time for the same product, in one process (medians of interleaved rounds).

    python scripts/gemm_study.py [T]        # T = tokens per GPU (default 16384 = 64 x 256)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402
from scripts.gemm_tune import timeit  # noqa: E402

dev = torch.device("cuda")


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    r = lambda *s: torch.randn(*s, device=dev).bfloat16()
    X, Wt, O, Wo, dY, dQKV = r(T, 640), r(1536, 640), r(T, 512), r(640, 512), r(T, 640), r(T, 1536)
    QKV, Y, dO = torch.empty(T, 1536, device=dev).bfloat16(), torch.empty(T, 640, device=dev).bfloat16(), \
        torch.empty(T, 512, device=dev).bfloat16()
    dW3, dWo = torch.empty(3, 640, 512, device=dev), torch.empty(512, 640, device=dev)
    bo = torch.randn(640, device=dev)
    cases = {
        "qkv fwd X.Wqkv^T [T,1536,640]": (2 * T * 1536 * 640, lambda t: hip.gemm(
            X, Wt, QKV, T, 512, 640, 640, 640, 1536, True, True, batch=3, sA=0, sB=512 * 640, sC=512, tile=t),
            lambda: torch.mm(X, Wt.t())),
        "out fwd O.Wo^T+b [T,640,512]": (2 * T * 640 * 512, lambda t: hip.gemm(
            O, Wo, Y, T, 640, 512, 512, 512, 640, True, True, bias=bo, tile=t),
            lambda: torch.addmm(bo.bfloat16(), O, Wo.t())),
        "dO = dY.Wo [T,512,640]": (2 * T * 640 * 512, lambda t: hip.gemm(
            dY, Wt[:512], dO, T, 512, 640, 640, 640, 512, True, True, tile=t),
            lambda: torch.mm(dY, Wt[:512].t())),
    }
    wgrad = {
        "dWqkv = X^T.dQKV [640,1536,T] f32": (2 * T * 640 * 1536, lambda t, sk: hip.gemm(
            X, dQKV, dW3, 640, 512, T, 640, 1536, 512, False, False, batch=3, sA=0, sB=512, sC=640 * 512,
            splitk=sk, tile=t, zero_c=True), lambda: torch.mm(X.t(), dQKV)),
        "dWo = O^T.dY [512,640,T] f32": (2 * T * 512 * 640, lambda t, sk: hip.gemm(
            O, dY, dWo, 512, 640, T, 512, 640, 640, False, False, splitk=sk, tile=t, zero_c=True),
            lambda: torch.mm(O.t(), dY)),
    }
    res = {}
    for name, (fl, f, blas) in cases.items():
        for t in (128, 1282, 1284, 2561, 12883, 12884):
            try:
                us = timeit(lambda: f(t))
            except Exception as e:  # noqa: BLE001
                print(name, t, "ERR", e)
                continue
            res[f"{name} tile{t}"] = (us, fl / us / 1e6)
        us = timeit(blas)
        res[f"{name} hipBLASLt"] = (us, fl / us / 1e6)
    for name, (fl, f, blas) in wgrad.items():
        for t in (1282, 1284, 12883, 12884):
            for sk in (1, 2, 4, 8, 16, 32):
                try:
                    us = timeit(lambda: f(t, sk))
                except Exception as e:  # noqa: BLE001
                    print(name, t, sk, "ERR", e)
                    continue
                res[f"{name} tile{t} sk{sk}"] = (us, fl / us / 1e6)
        us = timeit(blas)
        res[f"{name} hipBLASLt(bf16 out)"] = (us, fl / us / 1e6)
    for k, (us, tf) in res.items():
        print(f"{k:55s} {us:9.2f} us {tf:8.1f} TF/s", flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open(f"gpurun_out/gemm_study_T{T}.json", "w"), indent=1)


if __name__ == "__main__":
    main()
