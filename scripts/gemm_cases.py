"""The headline step's GEMM shapes (T = 16384 tokens) with their candidate tiles, timed in
interleaved rounds in one process (the case table scripts/gemm_ab.py times per library build).

    python scripts/gemm_cases.py [case ...]     cases: qkv qkv32 out dh dwqkv dwo (default: all)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402

dev = torch.device("cuda")
T = int(os.environ.get("T", "16384"))


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


def timeit_graph(fn, iters=20):
    """Launch-bound cases: ``iters`` calls captured in one HIP graph, timed over replays."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * iters) * 1e3


def cases():
    out = {}
    x = torch.randn(T, 640, device=dev).bfloat16()
    wqkv = torch.randn(3, 512, 640, device=dev).bfloat16()
    qkv = torch.empty(T, 1536, device=dev).bfloat16()

    def qkv_fn(tile):
        return lambda: hip.gemm(x, wqkv, qkv, T, 512, 640, 640, 640, 1536, True, True, batch=3, sA=0, sB=512 * 640,
                                sC=512, tile=tile)
    out["qkv"] = (qkv_fn, [2561, 2562], 2 * T * 640 * 1536)

    x32 = torch.randn(T, 640, device=dev)
    xb = torch.empty(T, 640, device=dev).bfloat16()

    def qkv32_fn(tile):
        if tile == "cast":   # the separate cast pass + the bf16 ping-pong GEMM
            return lambda: (hip.cast_into(x32, xb) if hasattr(hip, "cast_into") else xb.copy_(x32),
                            hip.gemm(xb, wqkv, qkv, T, 512, 640, 640, 640, 1536, True, True, batch=3, sA=0,
                                     sB=512 * 640, sC=512, tile=2561))
        return lambda: hip.gemm(x32, wqkv, qkv, T, 512, 640, 640, 640, 1536, True, True, batch=3, sA=0,
                                sB=512 * 640, sC=512, acopy=xb, tile=tile)
    out["qkv32"] = (qkv32_fn, [2561, "cast"], 2 * T * 640 * 1536)

    h = torch.randn(T, 512, device=dev).bfloat16()
    wo = torch.randn(640, 512, device=dev).bfloat16()
    bo = torch.randn(640, device=dev)
    y = torch.empty(T, 640, device=dev).bfloat16()
    ps = torch.empty(hip.psum_slots(T, 640), device=dev)

    def out_fn(tile):
        return lambda: hip.gemm(h, wo, y, T, 640, 512, 512, 512, 640, True, True, bias=bo, psum=ps, tile=tile)
    out["out"] = (out_fn, [1602], 2 * T * 512 * 640)

    dy = torch.randn(T, 640, device=dev).bfloat16()
    won = torch.randn(512, 640, device=dev).bfloat16()
    dh = torch.empty(T, 512, device=dev).bfloat16()

    def dh_fn(tile):
        return lambda: hip.gemm(dy, won, dh, T, 512, 640, 640, 640, 512, True, True, tile=tile)
    out["dh"] = (dh_fn, [2561, 1282], 2 * T * 512 * 640)

    dq = [torch.randn(T, 512, device=dev).bfloat16() for _ in range(3)]

    def dwqkv_fn(tile, S=8):
        if isinstance(tile, str):   # "tile:splits"
            tile, S = (int(v) for v in tile.split(":"))
        nkt = T // 64
        Se = hip.slab_count(nkt, S)
        sl = torch.empty(Se, 3, 640, 512, device=dev)
        return lambda: hip.gemm(x, dq[0], sl, 640, 512, T, 640, 512, 512, False, False, batch=3, sA=0,
                                sC=640 * 512, splitk=Se, tile=tile, slabs=True, b_list=dq)
    out["dwqkv"] = (dwqkv_fn, [1282], 2 * T * 640 * 1536)
    # ring depth / waves per CU at the weight-gradient shape ("tile:splits")
    out["dwqkv_ring"] = (dwqkv_fn, ["1282:8", "1284:8", "1284:4", "12883:8", "12883:4", "12884:8", "12884:4", "644:1", "644:2", "644:4", "1282:4"],
                         2 * T * 640 * 1536)

    def dwo_fn(tile, S=24):
        if isinstance(tile, str):
            tile, S = (int(v) for v in tile.split(":"))
        nkt = T // 64
        Se = hip.slab_count(nkt, S)
        sl = torch.empty(Se, 512, 640, device=dev)
        return lambda: hip.gemm(h, dy, sl, 512, 640, T, 512, 640, 640, False, False, sC=512 * 640, splitk=Se,
                                tile=tile, slabs=True)
    out["dwo"] = (dwo_fn, [1282], 2 * T * 512 * 640)
    out["dwo_ring"] = (dwo_fn, ["1282:24", "1284:24", "1284:12", "12883:24", "12883:12", "12884:24", "12884:12", "644:1", "644:2", "644:6", "644:8", "1282:12"],
                       2 * T * 512 * 640)

    # wider tiles at the weight-gradient shape (fewer operand bytes per FLOP, one block per CU):
    # 128x256 (12856, 3 stages), 256x128 (2563, 3 stages) -- and a 256x256 2-stage tile measured
    # in round 6 and removed (profiles/r6p_dw_wide_tiles.txt)
    out["dwqkv_wide"] = (dwqkv_fn, ["1282:6", "1282:8", "12856:4", "12856:6", "12856:8", "2563:4", "2563:6"],
                         2 * T * 640 * 1536)
    out["dwo_wide"] = (dwo_fn, ["1282:6", "1282:24", "12856:6", "12856:8", "12856:12", "2563:6", "2563:12"],
                       2 * T * 512 * 640)

    def dwgroup_fn(spec):
        # "tile0:S0/tile1:S1[:sep]": the dW_qkv batch and dW_o as one grouped grid (or separate)
        parts = spec.split("/")
        sep = parts[-1].endswith(":sep")
        (t0, S0), (t1, S1) = [(int(a), int(b)) for a, b, *_ in (q.split(":") for q in parts)]
        nkt = T // 64
        s0, s1 = hip.slab_count(nkt, S0), hip.slab_count(nkt, S1)
        sl0 = torch.empty(s0, 3, 640, 512, device=dev)
        sl1 = torch.empty(s1, 512, 640, device=dev)

        def run():
            if not sep:
                hip.gemm_group_begin()
            hip.gemm(x, dq[0], sl0, 640, 512, T, 640, 512, 512, False, False, batch=3, sA=0, sC=640 * 512,
                     splitk=s0, tile=t0, slabs=True, b_list=dq)
            hip.gemm(h, dy, sl1, 512, 640, T, 512, 640, 640, False, False, sC=512 * 640, splitk=s1, tile=t1,
                     slabs=True)
            if not sep:
                hip.gemm_group_end(sl0)
        return run
    out["dwgroup_big"] = (dwgroup_fn, ["1282:8/1282:24:sep", "1282:8/1282:24", "1282:6/1282:6", "1282:5/1282:7",
                                       "1282:6/1282:8", "1282:7/1282:5", "1282:8/1282:8", "1282:4/1282:4",
                                       "1282:6/1282:12", "1282:4/1282:12"],
                          2 * T * 640 * 1536 + 2 * T * 512 * 640)
    # one round of the 8-wave tiles at one block per CU (256 slots)
    out["dwgroup_8w"] = (dwgroup_fn, ["1282:6/1282:6", "12884:3/12884:3", "12883:3/12883:3", "12884:3/12884:3:sep",
                                      "12884:2/12884:6", "12883:2/12883:6"],
                          2 * T * 640 * 1536 + 2 * T * 512 * 640)
    out["dwgroup"] = (dwgroup_fn, ["12884:4/12884:12:sep", "12884:4/12884:12", "1282:4/1282:12", "12884:2/12884:6",
                                   "12884:3/12884:8", "1282:2/1282:6", "1282:8/1282:24", "12883:4/12883:12", "644:1/644:1:sep",
                                   "644:2/644:2:sep"],
                      2 * T * 640 * 1536 + 2 * T * 512 * 640)
    return out


_GRAPH_CASES = {"dwgroup", "dwgroup_big", "dwgroup_8w", "dwqkv_ring", "dwo_ring", "dwqkv_wide", "dwo_wide"}


def main():
    want = sys.argv[1:] or ["qkv", "qkv32", "out", "dh", "dwqkv", "dwo"]
    cs = cases()
    for name in want:
        mk, tiles, flops = cs[name]
        fns = {t: mk(t) for t in tiles}
        res = {t: [] for t in tiles}
        for _ in range(5):
            for t in tiles:
                res[t].append(timeit_graph(fns[t]) if name in _GRAPH_CASES else timeit(fns[t]))
        line = [f"{name:6s}"]
        for t in tiles:
            v = sorted(res[t])
            med = v[len(v) // 2]
            line.append(f"tile {t}: {med:7.2f} us ({flops / med / 1e6:6.0f} TF, min {v[0]:.2f})")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
