"""Device time of the attention kernels alone (forward, backward) at a given shape.

Each measurement replays a HIP graph of 20 back-to-back calls, so host launch cost is not
in the number (scripts/attn_bench.py times eager autograd calls, which are host-bound).

usage: python scripts/attn_time.py [B S H] ; prints one JSON line (microseconds per call)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402

B, S, H = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (64, 256, 8)
D, N = 64, 20
torch.manual_seed(0)
qkv = torch.randn(B, S, 3, H, D, device="cuda").bfloat16()
q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
scale = D ** -0.5
o, lse = hip.attn_fwd_lse(q, k, v, scale)
do = torch.randn_like(o)


def graph_time(fn):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(N):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    best = None
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1e3 / N
        best = t if best is None else min(best, t)
    return best


res = {"shape": [B, S, H, D],
       "fwd_us": round(graph_time(lambda: hip.attn_fwd_lse(q, k, v, scale)), 2),
       "bwd_us": round(graph_time(lambda: hip.attn_bwd_block(q, k, v, o, do, lse, scale)), 2)}
fl = 4.0 * B * H * S * S * D
res["fwd_TFLOPS"] = round(fl / (res["fwd_us"] * 1e-6) / 1e12, 1)
res["bwd_TFLOPS"] = round(2.5 * fl / (res["bwd_us"] * 1e-6) / 1e12, 1)
print(json.dumps(res), flush=True)
