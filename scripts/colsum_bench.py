"""Time ljs_colsum on [R][C] bf16 (column sums -> f32) and check it against torch.
LJS_COLSUM=0 selects the column-block ticket kernel, 1 (default) the full-row stream."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402


def main():
    for R, C in [(16384, 640), (2048, 640), (16384, 512), (16384, 2560)]:
        x = torch.randn(R, C, device="cuda").to(torch.bfloat16)
        out = torch.empty(C, device="cuda")
        ref = x.float().sum(0)
        hip.colsum(x, out)
        torch.cuda.synchronize()
        err = (out - ref).abs().max().item()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                hip.colsum(x, out)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 200
        print(f"colsum mode={os.environ.get('LJS_COLSUM', '1')} R={R} C={C}: {us:.2f} us "
              f"({R * C * 2 / us / 1e6:.2f} TB/s) max err {err:.3g}", flush=True)


if __name__ == "__main__":
    main()
