"""Per-kernel register / LDS / scratch use of the in-tree HIP library, from the code objects'
own AMDHSA metadata (what the compiler allocated), keyed by mangled kernel name.

rocprofv3's kernel table reports ``arch_vgpr_count`` from the kernel descriptor with the
pre-gfx950 4-register granule, i.e. HALF of what a gfx950 kernel allocates (the 256x128 QKV GEMM
shows 88 where the compiler's ``.vgpr_count`` is 143 and its allocation 176), and never the AGPRs
of the unified file.  ``scripts/kstats.py`` takes the true numbers from here instead.

    python scripts/kernel_resources.py [lib.so] [--grep gemm_dma]
"""
import argparse
import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIB = os.path.join(ROOT, "learning_jax_sharding_amd", "_lib", "libljs_kernels.so")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
_FIELDS = {".vgpr_count": "vgpr", ".agpr_count": "agpr", ".sgpr_count": "sgpr",
           ".vgpr_spill_count": "vgpr_spill", ".sgpr_spill_count": "sgpr_spill",
           ".group_segment_fixed_size": "lds", ".private_segment_fixed_size": "scratch"}


def _notes(co_path):
    out = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co_path], capture_output=True, text=True).stdout
    kernels, cur = {}, None
    for line in out.splitlines():
        s = line.strip()
        if s.startswith("- ."):          # a new kernel record starts with "- .<field>:"
            if cur and "name" in cur:
                kernels[cur["name"]] = cur
            cur = {}
            s = s[2:]
        if cur is None:
            continue
        m = re.match(r"(\.[a-z_]+):\s+(\S+)$", s)
        if not m:
            continue
        k, v = m.groups()
        if k == ".name":
            cur["name"] = v
        elif k in _FIELDS:
            try:
                cur[_FIELDS[k]] = int(v)
            except ValueError:
                pass
    if cur and "name" in cur:
        kernels[cur["name"]] = cur
    return kernels


def resources(lib=DEFAULT_LIB):
    """{mangled kernel name: {vgpr, agpr, sgpr, vgpr_spill, sgpr_spill, lds, scratch, alloc}};
    ``alloc`` = VGPRs + AGPRs rounded up to the 8-register gfx950 granule."""
    res = {}
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", lib, os.path.join(td, "x")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for i, s in enumerate(starts):
            e = starts[i + 1] if i + 1 < len(starts) else len(data)
            part = os.path.join(td, f"b{i}")
            with open(part, "wb") as f:
                f.write(data[s:e])
            co = os.path.join(td, f"co{i}.o")
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}", f"--output={co}"],
                               capture_output=True)
            if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            res.update(_notes(co))
    for k in res.values():
        tot = k.get("vgpr", 0) + k.get("agpr", 0)
        k["alloc"] = -(-tot // 8) * 8
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=DEFAULT_LIB)
    ap.add_argument("--grep", default="")
    a = ap.parse_args()
    for name, k in sorted(resources(a.lib).items()):
        if a.grep in name:
            print(f"{k.get('vgpr', 0):4d} v {k.get('agpr', 0):3d} a {k.get('sgpr', 0):3d} s  "
                  f"spill {k.get('vgpr_spill', 0)}/{k.get('sgpr_spill', 0)}  lds {k.get('lds', 0):6d}  {name}")


if __name__ == "__main__":
    main()
