"""Per-step duration beside the MEASURED shader clock (verdict r5 item 7: is the slow start of a
process a clock transient?).

Input: a rocprofv3 --kernel-trace database of ``LJS_CLOCK_PROBE=<json> python bench.py ...`` and
that json.  Steps are delimited by the probe kernel bench.py launches after every training step
(csrc/kernels/diag.hip); its record k holds the shader clock measured right after step k
(delta s_memtime / delta s_memrealtime x 100 MHz over a 3 us spin).

    python scripts/clock_ramp.py gpurun_out/r6b/ramp/run_results.db gpurun_out/r6b/clock.json [--out f.md]
"""
import argparse
import collections
import json
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("clock")
    ap.add_argument("--marker", default="clock_probe")
    ap.add_argument("--top", type=int, default=5)
    ap.add_argument("--out")
    a = ap.parse_args()
    clk = json.load(open(a.clock))
    recs = clk["records"]
    c = sqlite3.connect(a.db)
    ks = list(c.execute("select name, start, end from kernels order by start"))
    steps, cur = [], []
    for name, s, e in ks:
        if a.marker in name:
            steps.append(cur)
            cur = []
        else:
            cur.append((name, s, e))
    tot = collections.Counter()
    for st in steps[len(steps) // 2:]:
        for name, s, e in st:
            tot[name] += e - s
    heavy = [n for n, _ in tot.most_common(a.top)]

    def short(n):
        n = n.replace("(anonymous namespace)::", "").replace("void ", "")
        return n.split("(")[0][:26]

    lines = [f"source: `{a.db}` + `{a.clock}`: {len(steps)} steps delimited by the clock probe, "
             f"{len(recs)} clock records ({clk.get('warm_run')} untimed + {clk.get('steps')} timed steps); "
             "SCLK = delta s_memtime / delta s_memrealtime x 100 MHz, measured on the GPU after each step; us",
             "", "| step | SCLK MHz | wall | kernels | " + " | ".join(short(n) for n in heavy) + " |",
             "|---" * (4 + len(heavy)) + "|"]
    for i, st in enumerate(steps):
        if not st:
            continue
        busy = sum(e - s for _, s, e in st)
        wall = st[-1][2] - st[0][1]
        per = collections.Counter()
        for name, s, e in st:
            per[name] += e - s
        sclk = f"{recs[i]['sclk_mhz']:.0f}" if i < len(recs) else "-"
        lines.append(f"| {i} | {sclk} | {wall / 1e3:.1f} | {busy / 1e3:.1f} | "
                     + " | ".join(f"{per[n] / 1e3:.1f}" for n in heavy) + " |")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
