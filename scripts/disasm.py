"""Disassemble one kernel of the in-tree kernel library (gfx950 code object from .hip_fatbin).

    python scripts/disasm.py <substring of the mangled name> [lib]   -> stdout
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_resources import DEFAULT_LIB, LLVM, MAGIC  # noqa: E402


def main():
    pat, lib = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else DEFAULT_LIB)
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", lib, os.path.join(td, "x")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for i, s in enumerate(starts):
            e = starts[i + 1] if i + 1 < len(starts) else len(data)
            part, co = os.path.join(td, f"b{i}"), os.path.join(td, f"co{i}.o")
            open(part, "wb").write(data[s:e])
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}", f"--output={co}"],
                               capture_output=True)
            if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            syms = subprocess.run([f"{LLVM}/llvm-readelf", "-sW", co], capture_output=True, text=True).stdout.split()
            for name in syms:
                if pat in name and not name.endswith(".kd"):
                    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", f"--disassemble-symbols={name}",
                                          co], capture_output=True, text=True).stdout
                    print(out)
                    return


if __name__ == "__main__":
    main()
