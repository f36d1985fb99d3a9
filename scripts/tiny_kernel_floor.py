import sys, os, torch
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
from learning_jax_sharding_amd.ops import hip
from scripts.small_kernels import graph_time
g = torch.ones((), dtype=torch.bfloat16, device="cuda")
print("bcast_scalar", graph_time(lambda: hip.bcast_scalar(g, 640, 16384, True)))
p = torch.randn(2560, device="cuda")
o = torch.empty((), device="cuda")
print("sum_partials", graph_time(lambda: hip.lib().ljs_sum_partials(hip._p(p), 2560, hip._p(o), 0, hip._stream(o))))
x = torch.empty(64, device="cuda")
print("torch fill", graph_time(lambda: x.fill_(1.0)))
