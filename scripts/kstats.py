"""Per-kernel summary of a rocprofv3 --kernel-trace run (rocpd SQLite ``*_results.db`` or
``*_kernel_stats.csv``) as a markdown table.

    python scripts/kstats.py gpurun_out/prof6/run_results.db --steps 30 [--title ...] [--out profiles/x.md]

``--steps`` divides totals into per-step numbers (warmup + timed steps the profiled run executed).
"""
import argparse
import collections
import csv
import sqlite3


def load(path):
    rows = collections.defaultdict(list)
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        # workgroups = product over x/y/z of grid / workgroup extents (grid is in work-items)
        for name, dur, gx, gy, gz, wx, wy, wz, vgpr, agpr, lds in c.execute(
                "select name, duration, grid_x, grid_y, grid_z, workgroup_x, workgroup_y, workgroup_z, "
                "vgpr_count, accum_vgpr_count, lds_size from kernels"):
            wgs = (gx // max(1, wx)) * (max(1, gy) // max(1, wy)) * (max(1, gz) // max(1, wz))
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
    lines += [f"source: `{a.path}` (rocprofv3 --kernel-trace); per-step = total / {a.steps}", "",
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
