"""Build the gfx950 HIP kernel library (``_lib/libljs_kernels.so``) in-tree.

Every ``csrc/kernels/*.hip`` file is compiled with ``hipcc --offload-arch=gfx950`` (in
parallel) and linked into one shared library exposing a plain C ABI (``ljs_*``), loaded with
ctypes by :mod:`learning_jax_sharding_amd.ops.hip`.  No torch headers are involved, so a
rebuild takes seconds and the library does not depend on the torch ABI.  The C++ host
runtime (``csrc/runtime``) is built into ``_lib/libljs_runtime.so`` the same way.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
LIBDIR = os.path.join(PKG, "_lib")
ARCH = os.environ.get("LJS_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result"]


def _sources(sub):
    d = os.path.join(HERE, sub)
    return sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith((".hip", ".cpp")))


def _digest(files):
    h = hashlib.sha256()
    for f in files + [os.path.join(HERE, "kernels", "common.h")]:
        if os.path.exists(f):
            with open(f, "rb") as fh:
                h.update(fh.read())
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()[:16]


def _file_flags(src):
    """Per-file extra flags from a first-line ``// LJS_HIPCC_FLAGS: ...`` comment."""
    with open(src) as f:
        first = f.readline()
    tag = "LJS_HIPCC_FLAGS:"
    return first.split(tag, 1)[1].split() if tag in first else []


def _compile(src, obj, extra):
    cmd = [HIPCC] + FLAGS + extra + _file_flags(src) + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build_lib(name: str, sub: str, extra_link=(), force: bool = False, verbose: bool = True,
              libdir: str = None, defines=()) -> str:
    libdir = libdir or LIBDIR
    os.makedirs(libdir, exist_ok=True)
    srcs = _sources(sub)
    out = os.path.join(libdir, f"lib{name}.so")
    stamp = out + ".stamp"
    dig = _digest(srcs) + ("/" + " ".join(defines) if defines else "")
    if not force and os.path.exists(out) and os.path.exists(stamp) and open(stamp).read().strip() == dig:
        return out
    objdir = os.path.join(libdir, "obj", name)
    os.makedirs(objdir, exist_ok=True)
    extra = ["-I", os.path.join(HERE, "kernels")] + list(defines)
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs) or 1)) as ex:
        objs = list(ex.map(lambda s: _compile(s, os.path.join(objdir, os.path.basename(s) + ".o"), extra), srcs))
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs + list(extra_link)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed for {out}:\n{r.stderr}")
    # a kernel whose host launch stub was not emitted links fine but fails at dlopen: catch it here
    nm = subprocess.run(["nm", "-D", "--undefined-only", out], capture_output=True, text=True)
    missing = [l for l in nm.stdout.splitlines() if "__device_stub__" in l]
    if missing:
        raise RuntimeError(f"{out}: undefined kernel stubs (add explicit instantiations):\n" + "\n".join(missing))
    with open(stamp, "w") as f:
        f.write(dig)
    if verbose:
        print(f"[ljs build] {out} ({len(srcs)} sources)")
    return out


def build_all(force: bool = False, verbose: bool = True):
    paths = [build_lib("ljs_kernels", "kernels", force=force, verbose=verbose)]
    if os.path.isdir(os.path.join(HERE, "runtime")) and _sources("runtime"):
        paths.append(build_lib("ljs_runtime", "runtime", extra_link=["-L/opt/rocm/lib", "-lrccl", "-lamdhip64"],
                               force=force, verbose=verbose))
    return paths


def build_variant(tag: str, defines, verbose: bool = True) -> str:
    """An alternative build of the kernel library (A/B timing of a kernel variant): compiled with
    ``defines`` (e.g. ``-DLJS_ATTN_PK=0``) into ``_lib/variants/<tag>/``; load it with
    ``LJS_KERNELS_LIB=<path>``."""
    return build_lib("ljs_kernels", "kernels", libdir=os.path.join(LIBDIR, "variants", tag), defines=tuple(defines),
                     verbose=verbose)


if __name__ == "__main__":
    if "--variant" in sys.argv:
        i = sys.argv.index("--variant")
        print(build_variant(sys.argv[i + 1], sys.argv[i + 2:]))
    else:
        print(build_all(force="--force" in sys.argv))
