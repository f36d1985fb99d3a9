"""Phase timing of the fused attention backward (attn_bwd_fused_kernel) from shader-clock stamps
(LJS_ATTN_BWD_TRACE build):

    LJS_KERNELS_LIB=learning_jax_sharding_amd/_lib/variants/bwdtrace/libljs_kernels.so \\
        python scripts/attn_bwd_phases.py [B] [kvdma]

Per block (averaged over blocks and waves, shader-clock cycles): prologue (start -> first query
block's Q / dO / O and delta ready), each query block of the sweep, and the dK / dV epilogue;
plus how the blocks' start times spread (the second round of blocks starts when the first ends)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    if len(sys.argv) > 2 and sys.argv[2] == "kvdma":   # K / V by LDS-DMA beside the first block's
        hip.set_attention_bwd_kv_dma(True)
    H, S, D = 8, 256, 64
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(5)
    qkv = torch.randn(B, S, 3, H, D, generator=g).bfloat16().to(dev)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    do = torch.randn(B, S, H, D, generator=g).bfloat16().to(dev)
    o, lse = hip.attn_fwd_lse(q, k, v, 0.125)
    for _ in range(5):
        hip.attn_bwd_block(q, k, v, o, do, lse, 0.125)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        hip.attn_bwd_block(q, k, v, o, do, lse, 0.125)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    waves = 8
    trace = torch.zeros((B, H, waves, 8), dtype=torch.int64, device=dev)
    hip.lib().ljs_attn_set_trace(hip._p(trace))
    hip.attn_bwd_block(q, k, v, o, do, lse, 0.125)
    torch.cuda.synchronize()
    hip.lib().ljs_attn_set_trace(None)
    t = trace.cpu().double()
    ok = (t[..., 0] > 0) & (t[..., 7] > 0)
    print(f"B={B}: {B * H} blocks, backward {us:.1f} us; {int(ok.sum())} of {ok.numel()} (block, wave) records")
    names = ["prologue"] + [f"query block {i}" for i in range(4)]
    for i, n in enumerate(names):
        d = (t[..., i + 1] - t[..., i])[ok]
        print(f"  {n:14s} {d.mean().item():8.0f} cycles")
    d = (t[..., 7] - t[..., 5])[ok]
    print(f"  {'epilogue':14s} {d.mean().item():8.0f} cycles")
    span = (t[..., 7] - t[..., 0])[ok]
    print(f"  block span {span.mean().item():8.0f} cycles")
    st = t[..., 0][ok]
    en = t[..., 7][ok]
    print(f"  kernel span {(en.max() - st.min()).item():.0f} cycles; block starts: "
          f"first {0:.0f}, median {(st.median() - st.min()).item():.0f}, last {(st.max() - st.min()).item():.0f}")


if __name__ == "__main__":
    main()
