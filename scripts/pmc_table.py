"""Per-kernel PMC table (markdown) from the three rocprofv3 --pmc passes of a session
(pmc_summary.py outputs): MFMA busy, VALU / LDS / SALU per MFMA, the wave-cycle breakdown and the
LDS bank-conflict share.

    python scripts/pmc_table.py gpurun_out/r5j [--title ...] [--out profiles/x.md]

Pass 1: SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_ANY; pass 2: SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE; pass 3:
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM
SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM.  MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs).  SQ_INSTS_VALU counts the MFMAs too.
"""
import argparse
import collections
import os
import re


def load(f):
    d = collections.defaultdict(dict)
    cur = None
    if not os.path.exists(f):
        return d
    for line in open(f):
        if line.startswith("## "):
            cur = line[3:].strip()
            continue
        m = re.match(r"\s+(\S+)\s+total=\s*([\d.]+)\s+per-dispatch=\s*([\d.]+)", line)
        if m and cur:
            d[cur][m.group(1)] = float(m.group(3))
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--title", default="")
    ap.add_argument("--out")
    a = ap.parse_args()
    p1, p2, p3 = (load(os.path.join(a.dir, f"pmc_{i}.txt")) for i in (1, 2, 3))
    lines = [f"# {a.title}", ""] if a.title else []
    lines += ["| kernel | MFMA busy % | VALU/MFMA | LDS/MFMA | SALU/MFMA | wait (barrier/vmcnt) % | wait inst % | "
              "active % | LDS conflict % of LDS cycles |", "|---|---|---|---|---|---|---|---|---|"]
    for k, A in p1.items():
        mf = A.get("SQ_INSTS_MFMA", 0)
        if not mf:
            continue
        B, C = p2.get(k, {}), p3.get(k, {})
        grbm = B.get("GRBM_GUI_ACTIVE", 0)
        busy = 100 * B.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (grbm / 8 * 1024) if grbm else 0.0
        wc = A.get("SQ_WAVE_CYCLES", 1) or 1
        conf = 100 * C.get("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, C.get("SQ_LDS_IDX_ACTIVE", 1.0))
        lines.append(f"| `{k}` | {busy:.1f} | {A.get('SQ_INSTS_VALU', 0) / mf:.2f} | {A.get('SQ_INSTS_LDS', 0) / mf:.2f} | "
                     f"{B.get('SQ_INSTS_SALU', 0) / mf:.2f} | {100 * B.get('SQ_WAIT_ANY', 0) / wc:.1f} | "
                     f"{100 * A.get('SQ_WAIT_INST_ANY', 0) / wc:.1f} | {100 * A.get('SQ_ACTIVE_INST_ANY', 0) / wc:.1f} | "
                     f"{conf:.1f} |")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
