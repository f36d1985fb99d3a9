"""Where does an LDS-DMA GEMM wave spend its time?  Timeline stamps of gemm_dma_kernel.

Needs the instrumented variant library (``python -m learning_jax_sharding_amd.csrc.build
--variant gtrace -DLJS_GEMM_TRACE``); this script loads it itself.  Per wave the kernel records
s_memtime stamps at its start, around every K-tile wait (before the counted ``s_waitcnt vmcnt``,
after it, after the barrier) and at its end.  Printed per case, averaged over all waves:

* ``vm``   cycles waiting for this wave's own DMA pieces of the next tile (memory latency / rate)
* ``bar``  cycles waiting at the barrier for the other waves (skew, LDS reads of others)
* ``work`` cycles between one tile's barrier and the next tile's wait (fragment reads, MFMAs,
  DMA issue, epilogues)
* ``tail`` cycles from the last wait to the end (last MFMAs + the last epilogue)

    python scripts/gemm_trace.py [case ...]      cases: qkv out dh dwqkv dwo (default: all)
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
os.environ.setdefault("LJS_KERNELS_LIB", os.path.join(ROOT, "learning_jax_sharding_amd", "_lib", "variants", "gtrace",
                                                      "libljs_kernels.so"))

import ctypes  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from learning_jax_sharding_amd.ops import hip  # noqa: E402

dev = torch.device("cuda")
T = int(os.environ.get("T", "16384"))


def cases():
    x = torch.randn(T, 640, device=dev).bfloat16()
    wqkv = torch.randn(3, 512, 640, device=dev).bfloat16()
    qkv = torch.empty(T, 1536, device=dev).bfloat16()
    h = torch.randn(T, 512, device=dev).bfloat16()
    wo = torch.randn(640, 512, device=dev).bfloat16()
    y = torch.empty(T, 640, device=dev).bfloat16()
    dy = torch.randn(T, 640, device=dev).bfloat16()
    won = torch.randn(512, 640, device=dev).bfloat16()
    dh = torch.empty(T, 512, device=dev).bfloat16()
    dq = [torch.randn(T, 512, device=dev).bfloat16() for _ in range(3)]
    nkt = T // 64
    s8 = hip.slab_count(nkt, 8)
    s24 = hip.slab_count(nkt, 24)
    sl8 = torch.empty(s8, 3, 640, 512, device=dev)
    sl24 = torch.empty(s24, 512, 640, device=dev)
    return {
        "qkv": (lambda tile: hip.gemm(x, wqkv, qkv, T, 512, 640, 640, 640, 1536, True, True, batch=3, sA=0,
                                      sB=512 * 640, sC=512, tile=tile), 2561),
        "out": (lambda tile: hip.gemm(h, wo, y, T, 640, 512, 512, 512, 640, True, True, tile=tile), 1602),
        "dh": (lambda tile: hip.gemm(dy, won, dh, T, 512, 640, 640, 640, 512, True, True, tile=tile), 1282),
        "dwqkv": (lambda tile: hip.gemm(x, dq[0], sl8, 640, 512, T, 640, 512, 512, False, False, batch=3, sA=0,
                                        sC=640 * 512, splitk=s8, tile=tile, slabs=True, b_list=dq), 1282),
        "dwo": (lambda tile: hip.gemm(h, dy, sl24, 512, 640, T, 512, 640, 640, False, False, sC=512 * 640,
                                      splitk=s24, tile=tile, slabs=True), 1282),
    }


def analyse(buf, slots):
    """buf: [waves][slots] u64 (0 = unused)."""
    rows = []
    for w in buf:
        end = int(w[slots - 1])
        st = [int(v) for v in w[:slots - 1]]
        n = 0
        while n < len(st) and st[n]:
            n += 1
        if n < 4 or not end:
            continue
        start = st[0]
        waits = st[1:n]
        k = len(waits) // 3
        vm = bar = work = 0
        prev = start
        for i in range(k):
            a, b, c = waits[3 * i:3 * i + 3]
            work += a - prev
            vm += b - a
            bar += c - b
            prev = c
        rows.append((end - start, vm, bar, work, end - prev, k))
    return np.array(rows, dtype=np.float64)


def main():
    L = hip.lib()
    L.ljs_gemm_set_trace.argtypes = [ctypes.c_void_p]
    L.ljs_gemm_set_trace.restype = ctypes.c_int
    slots = L.ljs_gemm_set_trace(None)
    if slots <= 0:
        raise SystemExit("the loaded kernel library has no LJS_GEMM_TRACE instrumentation")
    want = sys.argv[1:] or ["qkv", "out", "dh", "dwqkv", "dwo"]
    cs = cases()
    for name in want:
        fn, tile = cs[name]
        for _ in range(3):
            fn(tile)
        torch.cuda.synchronize()
        nblk = 4096
        buf = torch.zeros(nblk * 8 * slots, dtype=torch.int64, device=dev)
        L.ljs_gemm_set_trace(ctypes.c_void_p(buf.data_ptr()))
        fn(tile)
        torch.cuda.synchronize()
        L.ljs_gemm_set_trace(None)
        b = buf.view(nblk * 8, slots).cpu().numpy().astype(np.uint64)
        r = analyse(b, slots)
        if not len(r):
            print(f"{name}: no stamps")
            continue
        tot, vm, bar, work, tail, k = r.mean(0)
        print(f"{name:6s} tile {tile}: waves {len(r)}  waits/wave {k:.1f}  cycles/wave {tot:9.0f}  "
              f"vm {vm / tot * 100:5.1f}%  bar {bar / tot * 100:5.1f}%  work {work / tot * 100:5.1f}%  "
              f"tail {tail / tot * 100:5.1f}%  | per wait: vm {vm / k:6.0f} bar {bar / k:6.0f} work {work / k:6.0f}",
              flush=True)
        # distribution of the per-wait vm stall over the waves (p10 / p50 / p90)
        q = np.percentile(r[:, 1] / r[:, 5], [10, 50, 90])
        qb = np.percentile(r[:, 2] / r[:, 5], [10, 50, 90])
        print(f"       vm/wait p10/50/90 {q[0]:.0f}/{q[1]:.0f}/{q[2]:.0f}   bar/wait {qb[0]:.0f}/{qb[1]:.0f}/{qb[2]:.0f}",
              flush=True)


if __name__ == "__main__":
    main()
