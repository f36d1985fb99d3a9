"""A/B timing of kernel-library builds at the headline step's GEMM shapes (T = 16384 tokens):
the default tile of each case from scripts/gemm_cases.py, medians of 7 rounds x 20 launches.
Run once per build (``LJS_KERNELS_LIB=<variant .so>``), interleaving the processes.

    python scripts/gemm_ab.py [case ...]     cases: qkv out dh dwqkv dwo, or case:tile (default: all)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gemm_cases as gb  # noqa: E402


def main():
    want = sys.argv[1:] or ["qkv", "out", "dh", "dwqkv", "dwo"]
    cs = gb.cases()
    tag = os.path.basename(os.path.dirname(os.environ.get("LJS_KERNELS_LIB", "default/x")))
    for spec in want:
        name, _, t = spec.partition(":")       # "qkv:2562" times that tile instead of the default
        mk, tiles, flops = cs[name]
        tile = int(t) if t else tiles[-1]
        fn = mk(tile)
        v = sorted(gb.timeit(fn) for _ in range(7))
        med = v[len(v) // 2]
        print(f"{tag:10s} {name:6s} tile {tile}: {med:7.2f} us ({flops / med / 1e6:6.0f} TF, min {v[0]:.2f})",
              flush=True)


if __name__ == "__main__":
    main()
