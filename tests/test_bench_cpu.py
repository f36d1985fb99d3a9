"""bench.py's JSON contract for every model family, on host devices (tiny shapes, no GPU)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--batch-per-gpu", "2", "--seq", "32", "--dim", "64", "--heads", "2", "--dim-head", "32",
        "--ff-dim", "128", "--steps", "2", "--warmup", "1", "--min-warmup", "0"]


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
    # the JSON 'warmup' is the number of untimed steps that actually ran
    assert rec["warmup"] == rec["config"]["warmup_steps_run"] and rec["warmup_requested"] == 1
    assert rec["value"] >= 0 and rec["ms_per_step"] > 0  # value is rounded: ~0 TFLOPS on host
    assert rec["config"]["global_batch"] == 2 and rec["config"]["seq_len"] == 32
    assert rec["config"]["parallelism"] == ("fsdp1" if model == "fsdp" else "dp1")


@pytest.mark.parametrize("gpus,mesh,par", [(2, "dp", "dp2"), (4, "dp", "dp4"), (4, "2d", "dp2xtp2"), (8, "dp", "dp8"),
                                           (8, "2d", "dp4xtp2")])
def test_bench_spawns_ranks(gpus, mesh, par):
    """`bench.py --gpus N` outside torchrun launches N rank processes (gloo host ranks here,
    RCCL on GPUs) and reports the N-rank job - it never silently runs one device."""
    env = dict(os.environ, LJS_PLATFORM="cpu")
    env.pop("LJS_NUM_DEVICES", None)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--mesh", mesh, *TINY],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == gpus and rec["n_devices"] == gpus
    assert rec["config"]["parallelism"] == par
    assert rec["config"]["global_batch"] == 2 * gpus  # weak scaling: batch-per-gpu x N
    assert rec["config"]["comm"].startswith("gloo")
    assert rec["dtype"] == "bf16"
    assert rec["warmup"] == rec["config"]["warmup_steps_run"]
    # value is the whole-job aggregate (the driver's contract); the per-GPU rate the metric names
    # is tflops_per_gpu = value / n_gpus
    assert abs(rec["value"] - rec["tflops_per_gpu"] * gpus) <= 1e-3 * gpus
    # which communication ran: backend, paths per collective shape (agreed by every rank), the
    # gradient buckets and the timed eager all-reduce of their size through each path
    det = rec["comm_detail"]
    assert det["backend"] == "gloo" and det["world"] == gpus and det["routes_agree_across_ranks"]
    assert det["rccl_nranks"] is None          # gloo ranks: no RCCL communicator exists
    assert det["routes"] and all(r["path"] == "torch-gloo" for r in det["routes"]), det["routes"]
    assert det["grad_buckets"] and all(b["bytes"] > 0 for b in det["grad_buckets"])
    probe = {p["path"]: p for p in det["all_reduce_probe"]}
    assert probe["torch-gloo"]["us_per_call"] > 0 and "skipped" in probe["rccl"] and "skipped" in probe["p2p"]
    assert probe["torch-gloo"]["bytes"] >= sum(b["bytes"] for b in det["grad_buckets"]) - 16
    assert det["p2p_fallbacks"] == []
    # the reference's 2-D DP x TP layout is timed in the same job under the default DP mesh
    if mesh == "dp":
        sec = rec["secondary"]
        assert sec["routes_agree_across_ranks"] and sec["comm_routes"]
        assert any(r["kind"] in ("all_gather", "all_to_all") for r in sec["comm_routes"])
        assert "error" not in sec, sec
        assert sec["mesh"] == [gpus // 2, 2] and sec["parallelism"] == f"dp{gpus // 2}xtp2"
        assert sec["ms_per_step"] > 0 and sec["comm"].startswith("gloo")
        for k in ("tflops_per_gpu", "graph_segments", "steps_per_graph", "warmup_steps_run"):
            assert k in sec, k
    else:
        assert "secondary" not in rec


@pytest.mark.parametrize("gpus", [2])
def test_bench_secondary_2d_two_ranks(gpus):
    """N=2: the secondary object is the (1, 2) mesh (the reference layout at two GPUs); the
    headline fields are unchanged and the line is still ONE JSON line."""
    env = dict(os.environ, LJS_PLATFORM="cpu")
    env.pop("LJS_NUM_DEVICES", None)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), *TINY],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["config"]["parallelism"] == "dp2" and rec["config"]["mesh"] == [2, 1]
    assert rec["secondary"]["mesh"] == [1, 2] and rec["secondary"]["parallelism"] == "dp1xtp2"
    assert "error" not in rec["secondary"]


def test_watchdog_on_fail_hook_reports_and_sets_exit():
    """A hang in a later phase runs the on_fail hook (bench.py prints the headline it already
    has) and exits with the hook's status; the per-phase deadline overrides the default."""
    import time
    from learning_jax_sharding_amd.comm.watchdog import CommWatchdog
    codes, seen = [], []
    wd = CommWatchdog(None, timeout_s=100.0, poll_s=0.01, exit_fn=codes.append, grace_s=0.0)
    wd.on_fail = lambda reason: seen.append(reason) or 0
    wd.start()
    wd.phase("secondary", 0.05)
    t0 = time.time()
    while not codes and time.time() - t0 < 5:
        time.sleep(0.01)
    wd.stop()
    assert codes == [0] and seen and "secondary" in seen[0]


def test_watchdog_on_fail_none_keeps_nonzero_exit():
    """bench.py's hook prints the headline and returns None: the watchdog's non-zero EXIT_CODE
    stands (a run that hung never exits 0), and a deadline lowered by ``phase`` is measured from
    that phase's own start."""
    import time
    from learning_jax_sharding_amd.comm.watchdog import EXIT_CODE, CommWatchdog
    codes, seen = [], []
    wd = CommWatchdog(None, timeout_s=100.0, poll_s=0.01, exit_fn=codes.append, grace_s=0.0)
    wd.on_fail = lambda reason: seen.append(reason)
    wd.start()
    time.sleep(0.1)
    wd.phase("secondary", 0.3)    # shorter than the time already spent in "startup": no false hang
    time.sleep(0.15)
    assert not codes
    t0 = time.time()
    while not codes and time.time() - t0 < 5:
        time.sleep(0.01)
    wd.stop()
    assert codes == [EXIT_CODE] and seen and "secondary" in seen[0]


def test_bench_min_warmup_counts_every_untimed_step():
    env = dict(os.environ, LJS_NUM_DEVICES="1")
    env.pop("LJS_PLATFORM", None)
    args = [a if a != "0" else "6" for a in TINY]  # --min-warmup 6
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["warmup"] == 6 == rec["config"]["warmup_steps_run"] and rec["warmup_requested"] == 1


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, LJS_PLATFORM="cpu", WORLD_SIZE="2", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", *TINY],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)


def test_bench_fp8_dtype_label():
    env = dict(os.environ, LJS_NUM_DEVICES="1", LJS_PLATFORM="cpu")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", "ff", "--fp8", *TINY],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    if r.returncode != 0 and "fp8" in r.stderr.lower() and "gpu" in r.stderr.lower():
        pytest.skip("MX-fp8 path needs the GPU")
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["dtype"] == "mx-fp8"
