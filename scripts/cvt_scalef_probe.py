"""Semantics probe of v_cvt_scalef32_pk_fp8_bf16 (gfx950 scaled fp8 conversion) against the
reference MX quantization path (bf16 -> f32, times 2^-x, RNE to e4m3): which scale argument
(2^x or 2^-x), if any, reproduces the reference bytes exactly.

usage: python scripts/cvt_scalef_probe.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.ops import hip  # noqa: E402


def main():
    n = 1 << 20
    g = torch.Generator(device="cpu").manual_seed(0)
    mag = torch.exp2(torch.randint(-20, 20, (n, 2), generator=g).float())
    v = (torch.randn(n, 2, generator=g) * mag).bfloat16()
    amax = v.float().abs().amax(1)
    m, e = torch.frexp(amax)
    x = (e - 1 - 8 + (m > 0.875).int()).clamp(-127, 127).int()
    words = v.view(torch.int16).to(torch.int32) & 0xFFFF
    packed = (words[:, 0] | (words[:, 1] << 16)).to(torch.int64)
    packed = torch.where(packed >= 2**31, packed - 2**32, packed).to(torch.int32).cuda()
    xs = x.cuda()
    out = torch.zeros(4 * n, dtype=torch.int32, device="cuda")
    lib = hip.lib()
    lib.ljs_debug_cvt_scalef.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p]
    rc = lib.ljs_debug_cvt_scalef(hip._p(packed), hip._p(xs), hip._p(out), n, hip._stream(out))
    assert rc == 0, rc
    torch.cuda.synchronize()
    o = out.view(n, 4).cpu().numpy()
    ref, up, dn = o[:, 0], o[:, 2], o[:, 3]
    print(f"scale=2^x  matches {np.mean(up == ref) * 100:.4f} %")
    print(f"scale=2^-x matches {np.mean(dn == ref) * 100:.4f} %")
    bad = np.nonzero(up != ref)[0][:5]
    for i in bad:
        print("  e.g.", v[i].float().tolist(), int(x[i]), hex(ref[i]), hex(up[i]), hex(dn[i]))


if __name__ == "__main__":
    main()
