"""The native libraries are built in-tree for gfx950 and export the full C ABI the Python
side binds (CPU: loading needs no GPU)."""
import ctypes
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "learning_jax_sharding_amd", "_lib")


def _exports(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


@pytest.fixture(scope="module")
def built():
    k = os.path.join(LIB, "libljs_kernels.so")
    r = os.path.join(LIB, "libljs_runtime.so")
    if not (os.path.exists(k) and os.path.exists(r)):
        from learning_jax_sharding_amd.csrc import build
        build.build_all()
    return k, r


def test_kernel_library_abi(built):
    from learning_jax_sharding_amd.ops.hip import _SIGS
    ex = _exports(built[0])
    missing = [n for n in list(_SIGS) + ["ljs_p2p_barrier", "ljs_p2p_reduce", "ljs_p2p_gather", "ljs_p2p_copy",
                                         "ljs_attn_set_bwd_fused", "ljs_gemm_mx_fp8", "ljs_quant_mx_rows"]
               if n not in ex]
    assert not missing, missing
    # every template kernel has its host launch stub (hipcc drops them without explicit instantiation)
    und = subprocess.run(["nm", "-D", "--undefined-only", built[0]], capture_output=True, text=True).stdout
    assert "__device_stub__" not in und


def test_runtime_library_abi(built):
    ex = _exports(built[1])
    for n in ("ljs_comm_init", "ljs_comm_split", "ljs_comm_async_error", "ljs_comm_abort", "ljs_comm_all_reduce",
              "ljs_comm_all_to_all", "ljs_p2p_alloc", "ljs_p2p_open", "ljs_p2p_enable_peer", "ljs_rt_device_info"):
        assert n in ex, n
    lib = ctypes.CDLL(built[1])
    assert lib.ljs_rt_version() == 1
    assert 0 < lib.ljs_rt_ipc_handle_size() <= 64


def test_gfx950_code_object(built):
    """The kernel library carries gfx950 machine code (not a generic/other-arch target)."""
    blob = open(built[0], "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
