"""Where the fused Q/K/V + attention forward differs from the separate kernels (debug aid)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for B, H, K in [(1, 1, 128), (2, 8, 640)]:
        T, N = B * 256, 64 * H
        g = torch.Generator(device="cpu").manual_seed(31)
        x = torch.randn(T, K, generator=g).bfloat16().to(dev)
        wt = (torch.randn(3, N, K, generator=g) * 0.05).bfloat16().to(dev).contiguous()
        out = torch.full((T, 3 * N), float("nan"), device=dev).bfloat16()
        scale = 64 ** -0.5
        o, lse = hip.qkv_attn_fwd(x, wt, out, H, scale)
        ref = torch.empty_like(out)
        hip.gemm(x, wt, ref, T, N, K, K, K, 3 * N, True, True, batch=3, sA=0, sB=N * K, sC=N)
        q, k, v = (ref.view(B, 256, 3, H, 64)[:, :, i] for i in range(3))
        o_ref, lse_ref = hip.attn_fwd_lse(q, k, v, scale)
        # fp32 torch reference
        qf, kf, vf = q.float(), k.float(), v.float()
        s = torch.einsum("bshd,bthd->bhst", qf, kf) * scale
        p = torch.softmax(s, -1).bfloat16().float()
        o_t = torch.einsum("bhst,bthd->bshd", p, vf)
        torch.cuda.synchronize()
        o4 = o.view(B, 256, H, 64).float()
        print(f"B={B} H={H} K={K}: qkv equal {torch.equal(out, ref)}; nan in o {torch.isnan(o4).any().item()}")
        d = (o4 - o_ref.float()).abs()
        print(f"  fused vs kernel: max {d.max().item():.3g}, rows differing {(d.amax(-1) > 0).sum().item()} of {B * 256 * H}")
        print(f"  fused vs torch {(o4 - o_t).abs().max().item():.3g}; kernel vs torch {(o_ref.float() - o_t).abs().max().item():.3g}")
        dl = (lse.view(B, H, 256) - lse_ref).abs()
        print(f"  lse max diff {dl.max().item():.3g}")
        bad = (d.amax(-1) > 0)   # [B, S, H]
        rows = bad.any(0).any(-1).nonzero().flatten().tolist()
        print(f"  differing query rows (any b, h): {rows[:40]}{' ...' if len(rows) > 40 else ''} ({len(rows)})")
        heads = bad.any(0).any(0).nonzero().flatten().tolist()
        print(f"  differing heads: {heads}")


if __name__ == "__main__":
    main()
