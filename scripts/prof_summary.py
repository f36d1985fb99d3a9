"""Summarise a rocprofv3 --kernel-trace --stats run into a markdown table (per-step us)."""
import csv
import sys


def main(stats_csv, steps, title, out):
    rows = list(csv.DictReader(open(stats_csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"# {title}", "", f"source: `{stats_csv}` (rocprofv3 --kernel-trace --stats); "
             f"per-step = total / {steps} profiled steps", "",
             "| kernel | calls | avg us | per-step us | % |", "|---|---|---|---|---|"]
    for r in rows:
        name = r["Name"].replace("(anonymous namespace)::", "").replace("|", "/")
        if len(name) > 80:
            name = name[:77] + "..."
        lines.append(f"| `{name}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | "
                     f"{float(r['TotalDurationNs'])/1e3/steps:.1f} | {float(r['Percentage']):.1f} |")
    lines.append(f"| **total GPU kernel time** | | | **{tot/1e3/steps:.1f}** | 100 |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4])
