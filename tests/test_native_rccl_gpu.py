"""Native RCCL rank communicators (comm/native.py RankRccl) on the one-GPU box.

A one-rank communicator is the only RCCL communicator one GPU admits, so this checks the
plumbing the 8-GPU run depends on: unique-id exchange through the torch.distributed store,
ncclCommInitRank / ncclCommSplit, every collective's buffer contract, and - the point of the
design - that the collectives are captured into a HIP graph and replay from it.  The
multi-rank code path of the whole training step is rehearsed separately with the 'fake'
backend (tests/test_rehearsal_gpu.py)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r'''
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["ROOT"])
dist.init_process_group("nccl", rank=0, world_size=1, init_method="tcp://127.0.0.1:29631",
                        device_id=torch.device("cuda", 0))
from learning_jax_sharding_amd.comm import native
assert native.rank_eligible()
rc = native.RankRccl(0, 1, 0)
h = rc.partition(((0,),))
assert h == rc._world_h
x = torch.arange(1024, device="cuda", dtype=torch.float32)
rc.all_reduce_(h, x)
assert torch.equal(x, torch.arange(1024, device="cuda", dtype=torch.float32))
xb = torch.randn(4096, device="cuda").bfloat16()
out = torch.empty_like(xb)
rc.all_gather(h, xb, out)
assert torch.equal(out, xb)
rs = torch.empty_like(xb)
rc.reduce_scatter(h, xb, rs)
assert torch.equal(rs, xb)
a2a = rc.all_to_all(h, xb, torch.empty_like(xb), 1)
assert torch.equal(a2a, xb)
# captured into a HIP graph: the all-reduce and the kernels around it replay together
buf = torch.zeros(1 << 20, device="cuda")
src = torch.ones(1 << 20, device="cuda")
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    g.capture_begin()
    buf.copy_(src)
    rc.all_reduce_(h, buf)
    buf.mul_(3.0)
    g.capture_end()
torch.cuda.current_stream().wait_stream(s)
for k in range(3):
    src.fill_(float(k + 1))
    g.replay()
    torch.cuda.synchronize()
    assert torch.all(buf == 3.0 * (k + 1)), (k, buf[:4])
rc.check()
print("native rccl ok")
dist.destroy_process_group()
'''


def test_rank_rccl_single_rank_and_graph_capture(tmp_path):
    script = tmp_path / "rr.py"
    script.write_text(_SCRIPT)
    env = dict(os.environ, ROOT=ROOT)
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "native rccl ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
