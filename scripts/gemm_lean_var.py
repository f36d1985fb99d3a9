"""Timing of the lean K-loop GEMM tiles at the step shapes for ONE kernel-library build (run once
per variant with LJS_KERNELS_LIB=..., interleaving the processes): medians of 7 x 20 launches.

    python scripts/gemm_lean_var.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gemm_lean_ab as g  # noqa: E402


def main():
    tag = os.path.basename(os.path.dirname(os.environ.get("LJS_KERNELS_LIB", "default/x")))
    for T in (16384, 2048):
        for name, mk, tiles, flops, outp in g.cases(T):
            for t in tiles:
                fn = mk(t + g.LEAN)
                v = sorted(g.timeit(fn) for _ in range(7))
                med = v[len(v) // 2]
                print(f"{tag:10s} T={T} {name:8s} tile {t}: {med:7.2f} us ({flops / med / 1e6:6.0f} TF, min {v[0]:.2f})",
                      flush=True)


if __name__ == "__main__":
    main()
