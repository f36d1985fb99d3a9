"""Multi-rank rehearsal on one GPU: the 'fake' torch.distributed backend lets ONE process play
rank 0 of an N-rank data-parallel job (every collective completes without moving data), so
the full N-GPU code path of bench.py - process groups, gradient buckets, collectives captured
inside the step's HIP graph, side-stream joins - runs on the one-GPU box.  Checks that it runs,
that the step is captured without cuts, and that its overhead over the 1-GPU step is small."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(env_extra, *args):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    env.pop("LJS_NUM_DEVICES", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


def test_dp8_rehearsal_single_graph():
    base = ("--steps", "30", "--warmup", "5", "--batch-per-gpu", "16")
    one = _bench({}, *base)
    reh = _bench({"WORLD_SIZE": "8", "RANK": "0", "LOCAL_RANK": "0", "LJS_DIST_BACKEND": "fake",
                  "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29641"}, "--gpus", "8", *base)
    assert reh["n_gpus"] == 8 and reh["config"]["parallelism"] == "dp8"
    assert reh["config"].get("graph_segments") == 1, reh["config"]
    # the DP machinery (bucketing, casts, captured collectives) costs little over one GPU
    assert reh["ms_per_step"] <= one["ms_per_step"] * 1.15 + 0.02, (reh["ms_per_step"], one["ms_per_step"])


def _bench_raw(env_extra, *args, timeout=300):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    env.pop("LJS_NUM_DEVICES", None)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        if k not in env_extra:
            env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          env=env, timeout=timeout)


def test_real_spawn_two_gloo_ranks_on_one_gpu():
    """The launcher the driver's scaling run uses (`bench.py --gpus N` -> torch.distributed.run
    child -> N ranks), exercised end to end on the one-GPU box: two ranks share GPU 0 over gloo
    (RCCL refuses two ranks on one GPU), so gradient all-reduces cut the captured step."""
    r = _bench_raw({"LJS_DIST_BACKEND": "gloo"}, "--gpus", "2", "--steps", "8", "--warmup", "2",
                   "--batch-per-gpu", "8")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["comm"].startswith("gloo")
    assert rec["config"]["graph_segments"] > 1, rec["config"]


def test_two_ranks_one_gpu_tp_p2p_single_graph():
    """The reference's model (TP) axis over two real ranks sharing GPU 0, every collective of the
    step (weight gathers, K/V gathers, the out-projection all-to-all, gradient reduce-scatters)
    through the IPC peer-memory kernels (LJS_P2P=1): bytes really move between the processes and
    the whole step is ONE captured graph (no gloo cut)."""
    r = _bench_raw({"LJS_DIST_BACKEND": "gloo", "LJS_P2P": "1", "LJS_P2P_MAX_KB": "65536", "LJS_COMM_TIMEOUT_S": "90"}, "--gpus", "2",
                   "--mesh", "1x2", "--steps", "8", "--warmup", "2", "--batch-per-gpu", "8", "--graph-steps", "1")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["n_gpus"] == 2 and rec["config"]["mesh"] == [1, 2]
    assert rec["config"]["graph_segments"] == 1, rec["config"]


def test_fake_8rank_2d_mesh_single_graph():
    """The reference's 2-D DP x TP layout at 8 ranks ((4, 2) mesh): every collective of the step
    (weight all-gathers, K/V gathers, out-projection all-to-all, gradient reductions) is captured
    into ONE graph."""
    rec = _bench({"WORLD_SIZE": "8", "RANK": "0", "LOCAL_RANK": "0", "LJS_DIST_BACKEND": "fake",
                  "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29642"}, "--gpus", "8", "--mesh", "2d",
                 "--steps", "16", "--warmup", "2", "--batch-per-gpu", "16")
    assert rec["n_gpus"] == 8 and rec["config"]["parallelism"] == "dp4xtp2"
    assert rec["config"].get("graph_segments") == 1, rec["config"]


def test_mse_loss_bench_line():
    rec = _bench({}, "--steps", "16", "--warmup", "2", "--loss", "mse")
    assert rec["config"]["loss"].startswith("mean") and rec["ms_per_step"] > 0


def test_launcher_and_rank_agree_on_gpu_count():
    """The launcher's sysfs GPU count (no HIP init) matches what a rank's torch sees."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ljs_bench", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    import torch
    n_sys = b._visible_gpu_count()
    print("sysfs GPUs:", n_sys, "torch GPUs:", torch.cuda.device_count())
    assert n_sys >= torch.cuda.device_count() >= 1
