"""Per-step kernel durations by step index from a rocprofv3 --kernel-trace database: where do the
first steps of a process lose their time (verdict r4 item 7, the "slow start")?

Steps are delimited by a marker kernel that runs once per train step (the fused Adam).  For each
step: the wall span from the end of the previous step's marker to the end of this one, the sum of
kernel durations inside it, and the durations of the heaviest kernels, so a ramp can be told apart
as (a) kernels running slower (clock, TLB / page first-touch, caches) or (b) gaps between kernels
(launch, graph replay).

    python scripts/step_ramp.py gpurun_out/r5a/ramp/run_results.db [--marker adam_multi] [--out f.md]
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="adam_multi")
    ap.add_argument("--top", type=int, default=6)
    ap.add_argument("--out")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ks = list(c.execute("select name, start, end from kernels order by start"))
    steps, cur = [], []
    for name, s, e in ks:
        cur.append((name, s, e))
        if a.marker in name:
            steps.append(cur)
            cur = []
    tot = collections.Counter()
    for st in steps[len(steps) // 2:]:
        for name, s, e in st:
            tot[name] += e - s
    heavy = [n for n, _ in tot.most_common(a.top)]

    def short(n):
        n = n.replace("(anonymous namespace)::", "").replace("void ", "")
        return n.split("(")[0][:28]

    lines = [f"source: `{a.db}`; {len(steps)} steps delimited by `{a.marker}`; us", "",
             "| step | wall | kernels | gaps | " + " | ".join(short(n) for n in heavy) + " |",
             "|---" * (4 + len(heavy)) + "|"]
    prev_end = None
    for i, st in enumerate(steps):
        busy = sum(e - s for _, s, e in st)
        start = st[0][1] if prev_end is None else prev_end
        wall = st[-1][2] - start
        prev_end = st[-1][2]
        per = collections.Counter()
        for name, s, e in st:
            per[name] += e - s
        lines.append(f"| {i} | {wall / 1e3:.1f} | {busy / 1e3:.1f} | {(wall - busy) / 1e3:.1f} | "
                     + " | ".join(f"{per[n] / 1e3:.1f}" for n in heavy) + " |")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
