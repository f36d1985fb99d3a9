"""bench.py's JSON contract for every model family, on host devices (tiny shapes, no GPU)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--batch-per-gpu", "2", "--seq", "32", "--dim", "64", "--heads", "2", "--dim-head", "32",
        "--ff-dim", "128", "--steps", "2", "--warmup", "1"]


@pytest.mark.parametrize("model", ["attention", "layer", "ff", "fsdp"])
def test_bench_json_contract(model):
    env = dict(os.environ, LJS_NUM_DEVICES="1")
    env.pop("LJS_PLATFORM", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", model, *TINY],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in rec, k
    assert rec["n_gpus"] == 1 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["value"] >= 0 and rec["ms_per_step"] > 0  # value is rounded: ~0 TFLOPS on host
    assert rec["config"]["global_batch"] == 2 and rec["config"]["seq_len"] == 32
    assert rec["config"]["parallelism"] == ("fsdp1" if model == "fsdp" else "dp1")
