"""Per-kernel roofline rows from ONE rocprofv3 ``--kernel-trace --pmc ... --output-format csv`` run.

Joins counter_collection.csv (one row per dispatch x counter) with kernel_trace.csv (durations) on
the dispatch id and prints, per kernel name: dispatches, mean duration, memory-side bytes, the
achieved HBM bandwidth, the L2 hit rate and the instruction mix.  Byte estimates follow
MI355X_MICROARCH's counter notes: a TCC_EA0_RDREQ is a 128-B line fill for 16-B/lane streaming
reads (FETCH_SIZE tallies it as 64 B, half the real traffic) and a TCC_EA0_WRREQ a 64-B write --
estimates, labelled as such.  Durations come from the counter run (kernels serialised by the
profiler), so they are indicative, not the headline's.

    python scripts/roofline.py 'gpurun_out/r6d/pmc_b64/**/' [--steps 6] [--top 14] [--out f.md]
"""
import argparse
import collections
import csv
import glob
import os

HBM_BPS = 8.0e12      # MI355X HBM3E peak (MI355X_MICROARCH)


def _rows(pattern, base):
    out = []
    for f in glob.glob(os.path.join(pattern, "**", base), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:44]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=0,
                    help="divide per-kernel totals by this many steps (0: per dispatch of each kernel)")
    ap.add_argument("--top", type=int, default=14)
    ap.add_argument("--out")
    a = ap.parse_args()
    dur = {}
    for r in _rows(a.dir, "*kernel_trace.csv"):
        dur[r.get("Dispatch_Id") or r.get("Correlation_Id")] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    seen = collections.defaultdict(set)
    for r in _rows(a.dir, "*counter_collection.csv"):
        name = short(r.get("Kernel_Name") or r.get("Kernel-Name") or "")
        did = r.get("Dispatch_Id") or r.get("Correlation_Id")
        cnt[name][r["Counter_Name"]] += float(r["Counter_Value"])
        seen[name].add(did)
    rows = []
    for name, cs in cnt.items():
        ids = seen[name]
        t = sum(dur.get(i, 0) for i in ids) * 1e-9          # s
        n = len(ids)
        rd = cs.get("TCC_EA0_RDREQ_sum", cs.get("TCC_EA0_RDREQ", 0.0)) * 128.0
        wr = cs.get("TCC_EA0_WRREQ_sum", cs.get("TCC_EA0_WRREQ", 0.0)) * 64.0
        hit = cs.get("TCC_HIT_sum", 0.0)
        miss = cs.get("TCC_MISS_sum", 0.0)
        rows.append(dict(name=name, n=n, t=t, rd=rd, wr=wr,
                         hit=hit / max(1.0, hit + miss), valu=cs.get("SQ_INSTS_VALU", 0.0),
                         mfma=cs.get("SQ_INSTS_MFMA", 0.0), salu=cs.get("SQ_INSTS_SALU", 0.0)))
    rows.sort(key=lambda r: -r["t"])
    tot_t = sum(r["t"] for r in rows)
    per = max(1, a.steps)
    if not a.steps:          # per dispatch: each kernel's totals over its own dispatch count
        for r in rows:
            for k in ("t", "rd", "wr"):
                r[k] /= max(1, r["n"])
        tot_t = sum(r["t"] for r in rows)
    unit = f"per-step values = totals / {per}" if a.steps else "values per dispatch of each kernel"
    cu = ("calls/step", "us/step") if a.steps else ("calls", "us/call")
    lines = [f"source: `{a.dir}` ({len(dur)} dispatches); {unit}; "
             "bytes are memory-side (EA) estimates: RDREQ x 128 B + WRREQ x 64 B",
             "",
             f"| kernel | {cu[0]} | {cu[1]} | % | HBM rd MB | HBM wr MB | GB/s | % of 8 TB/s | L2 hit | VALU/MFMA |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows[:a.top]:
        bw = (r["rd"] + r["wr"]) / max(1e-12, r["t"])
        vm = f"{r['valu'] / r['mfma']:.1f}" if r["mfma"] else "no MFMA"
        lines.append(f"| {r['name']} | {r['n'] / per:.1f} | {r['t'] * 1e6 / per:.1f} | "
                     f"{100 * r['t'] / max(1e-12, tot_t):.1f} | {r['rd'] / 1e6 / per:.1f} | "
                     f"{r['wr'] / 1e6 / per:.1f} | {bw / 1e9:.0f} | {100 * bw / HBM_BPS:.0f} | "
                     f"{100 * r['hit']:.0f}% | {vm} |")
    rd = sum(r["rd"] for r in rows)
    wr = sum(r["wr"] for r in rows)
    lines.append(f"| **all** | {sum(r['n'] for r in rows) / per:.0f} | {tot_t * 1e6 / per:.1f} | 100 | "
                 f"{rd / 1e6 / per:.1f} | {wr / 1e6 / per:.1f} | {(rd + wr) / max(1e-12, tot_t) / 1e9:.0f} | "
                 f"{100 * (rd + wr) / max(1e-12, tot_t) / HBM_BPS:.0f} | | |")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
