"""The native runtime's host logic (csrc/runtime/comm.cpp) under AddressSanitizer + UBSan.

``csrc/tests/runtime_host_test.cpp`` links comm.cpp against a host model of the RCCL / HIP
entry points it calls (communicators as heap objects, grouped collectives executed on host
buffers at ncclGroupEnd) and checks member ordering, split by colour / key, the offset
arithmetic of all-to-all / permute, error propagation and handle lifetimes; ASan watches every
access and LeakSanitizer every communicator / buffer.  Runs on the CPU (SURVEY §5 sanitizers;
GPU ASan is not available on this pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "learning_jax_sharding_amd", "csrc")


@pytest.fixture(scope="module")
def binary(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None or not os.path.exists("/opt/rocm/include/rccl/rccl.h"):
        pytest.skip("needs a host C++ compiler and the ROCm headers")
    out = str(tmp_path_factory.mktemp("asan") / "runtime_host_test")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           os.path.join(CSRC, "runtime", "comm.cpp"), os.path.join(CSRC, "tests", "runtime_host_test.cpp"), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    return out


def _run(binary, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    return subprocess.run([binary, *args], capture_output=True, text=True, timeout=120, env=env)


def test_runtime_host_logic_clean_under_asan(binary):
    r = _run(binary)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "runtime host test: ok" in r.stdout
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def test_asan_is_armed(binary):
    """Negative control: a deliberate heap overflow in the same binary is caught."""
    r = _run(binary, "--asan-selfcheck")
    assert r.returncode != 0 and "heap-buffer-overflow" in r.stderr, r.stderr[-2000:]
