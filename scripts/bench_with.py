"""Run bench.py with attention kernel switches set first (A/B of the test setters in ops/hip.py,
which are not environment knobs):

    python scripts/bench_with.py bwd_fused=0 -- --steps 20 --warmup 5
    python scripts/bench_with.py qkv_gate=1 -- --batch-per-gpu 16   (fused projection at any item count)
"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    sets, rest = argv[:cut], argv[cut + 1:]
    from learning_jax_sharding_amd.ops import hip
    fns = {"bwd_fused": hip.set_attention_bwd_fused, "bwd_kv_dma": hip.set_attention_bwd_kv_dma,
           "dkv32": hip.set_attention_dkv32, "dq32": hip.set_attention_dq32, "bwd_pair": hip.set_attention_bwd_pair}
    for s in sets:
        k, v = s.split("=")
        if k == "qkv_gate":   # the fused projection + attention's items-per-CU gate: items >= v
            from learning_jax_sharding_amd.ops import linear
            linear._cu_count = lambda dev, _v=int(v): _v
            continue
        fns[k](bool(int(v)))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.argv = [os.path.join(root, "bench.py")] + rest
    runpy.run_path(sys.argv[0], run_name="__main__")


if __name__ == "__main__":
    main()
