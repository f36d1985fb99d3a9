"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel (sum over dispatches)."""
import collections
import csv
import glob
import sys


def main(pattern, out=None):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.Counter()
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("KernelName")
            name = name.replace("(anonymous namespace)::", "")[:60]
            agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Counter_Name"] == sorted(agg[name])[0]:
                pass
            calls[(name, r["Counter_Name"])] += 1
    lines = []
    for name, cs in sorted(agg.items(), key=lambda kv: -max(kv[1].values())):
        lines.append(f"## {name}")
        for c, v in sorted(cs.items()):
            n = calls[(name, c)]
            lines.append(f"  {c:28s} total={v:14.0f}  per-dispatch={v / max(1, n):14.1f}")
    txt = "\n".join(lines)
    print(txt)
    if out:
        open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
