"""Ring attention forward + backward on a 1 x N virtual mesh over one MI355X, for a kernel trace
showing each hop's K/V copies (side stream) concurrent with the flash-attention blocks.

    rocprofv3 --kernel-trace -d gpurun_out/ring -o ring -- python scripts/ring_trace.py
"""
import os
import sys
import time

os.environ.setdefault("LJS_PLATFORM", "gpu")
os.environ.setdefault("LJS_NUM_DEVICES", "4")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import learning_jax_sharding_amd as ljs  # noqa: E402
from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh  # noqa: E402
from learning_jax_sharding_amd.parallel import sequence as SQ  # noqa: E402
from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P  # noqa: E402
from learning_jax_sharding_amd.spmd.api import _fresh_leaf  # noqa: E402


def main():
    n = ljs.device_count()
    B, S, H = int(os.environ.get("B", "4")), int(os.environ.get("S", "8192")), 8
    mesh = Mesh(create_device_mesh((1, n)), ("data", "model"))
    sh = NamedSharding(mesh, P("data", "model"))
    g = torch.Generator().manual_seed(0)
    arrs = [ljs.device_put(torch.randn(B, S, H, 64, generator=g).bfloat16(), sh) for _ in range(3)]
    for mode in ("ring", "allgather"):
        for it in range(4):
            leaves = [_fresh_leaf(a) for a in arrs]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = SQ.context_parallel_attention(*leaves, mode=mode)
            outs = list(out.local.values())
            ins = [t for l in leaves for t in l.local.values()]
            torch.autograd.grad(outs, ins, [torch.ones_like(t) for t in outs])
            torch.cuda.synchronize()
            if it == 3:
                print(f"{mode}: fwd+bwd {1e3 * (time.perf_counter() - t0):.2f} ms (B={B} S={S} H={H}, 1x{n} mesh)",
                      flush=True)


if __name__ == "__main__":
    main()
