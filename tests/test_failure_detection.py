"""Failure detection on the RCCL path and the HIP-free multi-GPU launcher, on CPU.

The native runtime is replaced by a fake ctypes-like object, so the real RankRccl / CommWatchdog
code runs: an injected asynchronous RCCL error (or a phase that overruns its deadline while the
main thread is blocked, as in a device synchronize on a lost peer) must abort every communicator,
print a diagnosis naming the partition, and end the process non-zero within the deadline."""
import argparse
import os
import subprocess
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_FAKE = textwrap.dedent("""
    import sys, time
    sys.path.insert(0, {root!r})
    from learning_jax_sharding_amd.comm import native
    from learning_jax_sharding_amd.comm.watchdog import CommWatchdog

    class FakeRuntime:
        def __init__(self, fail_after):
            self.t0, self.fail_after, self.aborted = time.monotonic(), fail_after, []
        def ljs_comm_async_error(self, h):
            if self.fail_after is not None and time.monotonic() - self.t0 > self.fail_after and h == 0x22:
                return 6            # ncclRemoteError: a peer went away
            return 0
        def ljs_comm_error_string(self, rc):
            return b"remote process exited or there was a network error"
        def ljs_comm_abort(self, h):
            self.aborted.append(h)
            print(f"abort {{h:#x}}", flush=True)
            return 0
        def ljs_comm_destroy(self, h):
            return 0

    fake = FakeRuntime({fail_after})
    native.runtime = lambda: fake
    r = object.__new__(native.RankRccl)
    r.rank, r.world, r.device = 1, 4, 0
    r._world_h = 0x11
    r._parts = {{((0, 1), (2, 3)): 0x22}}
    r._log = {{}}
    r._note(0x11, "all_reduce", 5 << 20)
    r._note(0x22, "all_gather", 1 << 20)

    class Comm:
        _native = r

    wd = CommWatchdog(Comm(), timeout_s={timeout}, poll_s=0.05, grace_s=0.2).start()
    wd.phase("timed steps")
    time.sleep(60)   # the main thread is stuck (a device synchronize on a dead peer)
    print("not reached", flush=True)
""")


def _run(fail_after, timeout):
    src = _FAKE.format(root=ROOT, fail_after=fail_after, timeout=timeout)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", src], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, RANK="1"))
    return r, time.monotonic() - t0


def test_async_rccl_error_aborts_and_exits_nonzero():
    r, dt = _run(fail_after=0.3, timeout=30)
    from learning_jax_sharding_amd.comm.watchdog import EXIT_CODE
    assert r.returncode == EXIT_CODE, (r.returncode, r.stdout, r.stderr)
    assert dt < 20, dt
    assert "asynchronous RCCL error" in r.stderr and "(2, 3)" not in r.stdout
    assert "partition [[0, 1], [2, 3]] (this rank's group [0, 1])" in r.stderr, r.stderr
    assert "all_reduce x1 (5.24 MB/call)" in r.stderr, r.stderr
    assert "abort 0x11" in r.stdout and "abort 0x22" in r.stdout
    assert "not reached" not in r.stdout


def test_hang_past_deadline_exits_nonzero():
    r, dt = _run(fail_after=None, timeout=1.0)
    from learning_jax_sharding_amd.comm.watchdog import EXIT_CODE
    assert r.returncode == EXIT_CODE, (r.returncode, r.stdout, r.stderr)
    assert dt < 20, dt
    assert "deadline" in r.stderr and "'timed steps'" in r.stderr
    assert "not reached" not in r.stdout


def test_watchdog_quiet_when_healthy():
    from learning_jax_sharding_amd.comm.watchdog import CommWatchdog
    exits = []
    wd = CommWatchdog(None, timeout_s=5, poll_s=0.01, exit_fn=exits.append).start()
    for i in range(5):
        wd.phase(f"step {i}")
        time.sleep(0.02)
    wd.stop()
    assert exits == [] and wd.failed is None


def test_rank_rccl_close_destroys_every_communicator(monkeypatch):
    from learning_jax_sharding_amd.comm import native
    destroyed = []

    class RT:
        def ljs_comm_destroy(self, h):
            destroyed.append(h)
            return 0
    monkeypatch.setattr(native, "runtime", lambda: RT())
    r = object.__new__(native.RankRccl)
    r.rank, r.world, r.device = 0, 8, 0
    r._world_h, r._parts, r._log = 0x10, {((0, 1, 2, 3), (4, 5, 6, 7)): 0x20, ((0,), (1,)): None}, {}
    r.close()
    assert destroyed == [0x20, 0x10] and r._world_h is None and not r._parts


# ----------------------------------------------------------------------------- launcher
def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("ljs_bench", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_launcher_counts_gpus_without_torch(monkeypatch):
    b = _bench_module()
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert b._visible_gpu_count() == 0
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1")
    assert b._visible_gpu_count() <= 2


def test_launcher_refuses_missing_gpus_without_touching_torch():
    """No GPU here: `bench.py --gpus 2` (GPU platform) fails fast in the launcher, which never
    imports torch (checked by making `import torch` fail in the launcher process)."""
    env = dict(os.environ)
    for k in ("LJS_PLATFORM", "LJS_DIST_BACKEND", "WORLD_SIZE"):
        env.pop(k, None)
    code = ("import sys; sys.modules['torch'] = None; sys.argv = ['bench.py', '--gpus', '2'];"
            f"sys.path.insert(0, {ROOT!r}); import runpy; runpy.run_path({os.path.join(ROOT, 'bench.py')!r}, "
            "run_name='__main__')")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "needs 2 visible GPUs" in r.stderr


def test_bench_rejects_unsupported_head_dim_on_gpu():
    b = _bench_module()
    a = argparse.Namespace(model="attention", dim_head=128, mesh="dp", loss="sum", mode="train")
    with pytest.raises(SystemExit, match="dim-head 128"):
        b.check_args(a, on_gpu=True)
    b.check_args(a, on_gpu=False)          # host devices run any head dim (torch path)
    b.check_args(argparse.Namespace(model="attention", dim_head=64, mesh="dp", loss="sum", mode="train"), True)
    with pytest.raises(SystemExit, match="fsdp"):
        b.check_args(argparse.Namespace(model="fsdp", dim_head=64, mesh="2d", loss="sum", mode="train"), False)
