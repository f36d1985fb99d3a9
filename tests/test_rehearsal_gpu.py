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
