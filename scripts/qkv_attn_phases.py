"""Phase timing of the fused Q/K/V + attention forward kernel (qkv_attn_fwd_kernel) from its
shader-clock stamps: run with a LJS_QA_TRACE build,

    LJS_KERNELS_LIB=learning_jax_sharding_amd/_lib/variants/qatrace/libljs_kernels.so \\
        python scripts/qkv_attn_phases.py [B]

Per item (averaged over blocks and waves, in shader-clock cycles): K-loop (item start -> last
MFMAs issued), epilogue (-> images written, barrier passed), attention (-> O stored), and the gap
from one item's end to the next item's start."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    H, K = 8, 640
    T, N = B * 256, 64 * H
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(T, K, generator=g).bfloat16().to(dev)
    wt = (torch.randn(3, N, K, generator=g) * 0.05).bfloat16().to(dev).contiguous()
    out = torch.empty((T, 3 * N), dtype=torch.bfloat16, device=dev)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    trace = torch.zeros((cus, 8, 8, 4), dtype=torch.int64, device=dev)
    for _ in range(5):
        hip.qkv_attn_fwd(x, wt, out, H, 0.125)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        hip.qkv_attn_fwd(x, wt, out, H, 0.125)
    e1.record()
    trace.zero_()
    hip.qkv_attn_fwd(x, wt, out, H, 0.125, trace=trace)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    tr = trace.cpu()
    items = (T // 256) * H
    per_block = -(-items // cus)
    print(f"B={B}: {items} items on {min(cus, items)} blocks ({per_block} per block), kernel {us:.1f} us")
    names = ["K-loop", "epilogue", "attention"]
    nb = min(cus, items)
    for k in range(min(per_block, 8)):
        t = tr[:nb, :, k].double()
        ok = (t > 0).all(-1)
        if not ok.any():
            continue
        d = [(t[..., i + 1] - t[..., i])[ok].mean().item() for i in range(3)]
        line = f"  item {k}: " + ", ".join(f"{n} {v:8.0f}" for n, v in zip(names, d))
        if k + 1 < per_block:
            t2 = tr[:nb, :, k + 1].double()
            ok2 = ok & (t2[..., 0] > 0)
            if ok2.any():
                line += f", gap to next {(t2[..., 0] - t[..., 3])[ok2].mean().item():8.0f}"
        print(line + " cycles")
    t = tr[:nb].double()
    first = t[:, :, 0, 0][t[:, :, 0, 0] > 0]
    last = t[..., 3].amax(-1)
    last = last[last > 0]
    print(f"  span first stamp -> last stamp: {(last.max() - first.min()).item():.0f} cycles; "
          f"block spans {(t[..., 3].amax(-1) - t[:, :, 0, 0]).mean().item():.0f} mean")


if __name__ == "__main__":
    main()
