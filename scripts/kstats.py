"""Per-kernel summary of a rocprofv3 --kernel-trace run (rocpd SQLite ``*_results.db`` or
``*_kernel_stats.csv``) as a markdown table.

    python scripts/kstats.py gpurun_out/prof6/run_results.db --steps 30 [--title ...] [--out profiles/x.md]

``--steps`` divides totals into per-step numbers (warmup + timed steps the profiled run executed).
"""
import argparse
import collections
import csv
import sqlite3


def _true_regs():
    """mangled name -> compiler register use of the in-tree library (scripts/kernel_resources.py):
    rocprofv3 decodes gfx950 descriptors with the old 4-register granule (half the real count)."""
    try:
        import os
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from kernel_resources import resources
        return resources()
    except Exception:
        return {}


def load(path):
    rows = collections.defaultdict(list)
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        regs = _true_regs()
        # workgroups = product over x/y/z of grid / workgroup extents (grid is in work-items)
        for name, dur, gx, gy, gz, wx, wy, wz, vgpr, agpr, lds, mang in c.execute(
                "select K.name, K.duration, K.grid_x, K.grid_y, K.grid_z, K.workgroup_x, K.workgroup_y, "
                "K.workgroup_z, K.vgpr_count, K.accum_vgpr_count, K.lds_size, S.kernel_name from kernels K "
                "left join rocpd_info_kernel_symbol S on S.id = K.kernel_id and S.guid = K.guid"):
            wgs = (gx // max(1, wx)) * (max(1, gy) // max(1, wy)) * (max(1, gz) // max(1, wz))
            r = regs.get((mang or "").replace(".kd", ""))
            if r is not None:
                vgpr, agpr = f"{r.get('vgpr', 0)}", f"{r.get('agpr', 0)}"
            else:
                vgpr, agpr = f"~{2 * vgpr}", f"{agpr}"   # rocprof's descriptor count x 2 (gfx950 granule)
            rows[name].append((dur / 1e3, wgs, vgpr, agpr, lds))
    else:
        for r in csv.DictReader(open(path)):
            rows[r["Name"]].append((float(r["AverageNs"]) / 1e3, 0, 0, 0, 0))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--title", default="")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = load(a.path)
    total = sum(sum(d[0] for d in v) for v in rows.values())
    lines = []
    if a.title:
        lines += [f"# {a.title}", ""]
    lines += [f"source: `{a.path}` (rocprofv3 --kernel-trace); per-step = total / {a.steps}; VGPR/AGPR from the "
              "code objects' metadata (scripts/kernel_resources.py; '~' = rocprof's descriptor count x 2)", "",
              "| kernel | calls | avg us | per-step us | % | grid (WGs) | VGPR/AGPR | LDS B |",
              "|---|---|---|---|---|---|---|---|"]
    for name, v in sorted(rows.items(), key=lambda kv: -sum(d[0] for d in kv[1])):
        t = sum(d[0] for d in v)
        nm = name.replace("(anonymous namespace)::", "")
        if len(nm) > 90:
            nm = nm[:87] + "..."
        g = v[-1]
        lines.append(f"| `{nm}` | {len(v)} | {t / len(v):.2f} | {t / a.steps:.1f} | {100 * t / total:.1f} | "
                     f"{g[1]} | {g[2]}/{g[3]} | {g[4]} |")
    lines.append(f"| **total GPU kernel time** | | | **{total / a.steps:.1f}** | 100 | | | |")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
