"""What bounds the fused multi-tensor Adam (verdict r4 item 3: 20.8 us at B=64, 17 us at B=8)?
The step's parameter set (3 x [640, 512] QKV projections whose gradient is the 8 split-K slabs of
one batched slab GEMM, W_o [512, 640] with 24 slabs, 4 biases) timed in isolation with parts of
the work removed: slabs -> one plain gradient, shadows off, fewer slabs; and a torch copy of the
same byte count as a bandwidth yardstick.

    python scripts/adam_probe.py          (LJS_ADAM_THREADS=256|512|1024 picks the kernel form)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip, shadow  # noqa: E402

dev = torch.device("cuda")
ROUNDS = int(os.environ.get("ROUNDS", "7"))


_GRAPHS = {}


def timeit(fn, iters=20):
    # captured in a HIP graph: the host side of adam_multi (its tensor table) takes longer than
    # the kernel, so eager back-to-back launches would time the host
    g = _GRAPHS.get(fn)
    if g is None:
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        _GRAPHS[fn] = g
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def params(shadows: bool):
    ws = [torch.randn(640, 512, device=dev) * 0.02 for _ in range(3)] + [torch.randn(512, 640, device=dev) * 0.02]
    bs = [torch.zeros(512, device=dev) for _ in range(3)] + [torch.zeros(640, device=dev)]
    if shadows:
        for w in ws:
            shadow.get(w, "T")
            shadow.get(w, "N")
    st = [(torch.zeros_like(p), torch.zeros_like(p)) for p in ws + bs]
    return ws, bs, st


def entries(ws, bs, st, Sq, So):
    out = []
    gq = torch.randn(max(Sq, 1), 3, 640, 512, device=dev) * 1e-3
    go = torch.randn(max(So, 1), 512, 640, device=dev) * 1e-3
    for i in range(3):
        g = hip.SlabGrad(gq, Sq, i * 640 * 512, 512, 3 * 640 * 512, (640, 512)) if Sq else gq[0, i].contiguous()
        out.append((ws[i], g, *st[i]))
    g = hip.SlabGrad(go, So, 0, 640, 512 * 640, (512, 640)) if So else go[0].contiguous()
    out.append((ws[3], g, *st[3]))
    for i, b in enumerate(bs):
        out.append((b, torch.randn_like(b) * 1e-3, *st[4 + i]))
    return out


def main():
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    variants = {}
    nbytes = {}
    P = 3 * 640 * 512 + 512 * 640
    for name, sh, Sq, So in (("slabs 8/24 + shadows (step)", True, 8, 24), ("slabs 8/24, no shadows", False, 8, 24),
                             ("slabs 4/4 + shadows", True, 4, 4), ("slabs 2/2 + shadows", True, 2, 2),
                             ("plain grad + shadows", True, 0, 0), ("plain grad, no shadows", False, 0, 0)):
        ws, bs, st = params(sh)
        e = entries(ws, bs, st, Sq, So)
        variants[name] = (lambda e=e: hip.adam_multi(e, step, 1e-4, 0.9, 0.999, 1e-8, 0.0, increment_step=True))
        slab = 4 * (Sq * 3 * 640 * 512 + So * 512 * 640) if Sq else 4 * P
        nbytes[name] = slab + 24 * P + (8 * P if sh else 0)
    ws, bs, st = params(False)
    e = entries(ws, bs, st, 0, 0)
    variants["plain, no shadows, no ticket"] = (lambda e=e: hip.adam_multi(e, step, 1e-4, 0.9, 0.999, 1e-8, 0.0))
    nbytes["plain, no shadows, no ticket"] = 4 * P + 24 * P
    def sep(e=e):
        hip.adam_multi(e, step, 1e-4, 0.9, 0.999, 1e-8, 0.0)
        step.add_(1)
    variants["plain, no shadows, separate +1"] = sep
    nbytes["plain, no shadows, separate +1"] = 4 * P + 24 * P
    # size sweep of the plain-gradient form: fixed cost vs per-byte cost
    for f in (0.25, 0.5, 2, 4):
        R = int(640 * f)
        ps = [torch.randn(R, 512, device=dev) for _ in range(4)]
        e = [(q, torch.randn_like(q) * 1e-3, torch.zeros_like(q), torch.zeros_like(q)) for q in ps]
        name = f"plain, no shadows, x{f} size"
        variants[name] = (lambda e=e: hip.adam_multi(e, step, 1e-4, 0.9, 0.999, 1e-8, 0.0, increment_step=True))
        nbytes[name] = 4 * R * 512 * 4 * 7
    n = 50 << 20
    src, dst = torch.empty(n // 4, device=dev), torch.empty(n // 4, device=dev)
    variants["torch copy 50 MB -> 50 MB"] = lambda: dst.copy_(src)
    nbytes["torch copy 50 MB -> 50 MB"] = 2 * n
    res = {k: [] for k in variants}
    for _ in range(ROUNDS):
        for k, f in variants.items():
            res[k].append(timeit(f))
    print(f"LJS_ADAM_THREADS={os.environ.get('LJS_ADAM_THREADS', '256')}", flush=True)
    for k, v in res.items():
        v = sorted(v)
        med = v[len(v) // 2]
        print(f"{k:30s} {med:7.2f} us  {nbytes[k] / 1e6:6.1f} MB  {nbytes[k] / med / 1e6:5.2f} TB/s (min {v[0]:.2f})",
              flush=True)


if __name__ == "__main__":
    main()
