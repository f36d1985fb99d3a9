"""Which kernels ran concurrently with kernels of another HIP stream, from a rocprofv3
``--kernel-trace`` database: per kernel name on the non-dominant streams, the time it spent
overlapped with the dominant (main) stream's kernels, and what those were.

    python scripts/overlap_report.py gpurun_out/x/prof/run_results.db [--last N] [--out profiles/x.md]

``--last N``: only the last N dispatches (the timed steps) are considered.
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--out", default="")
    ap.add_argument("--title", default="kernel overlap across HIP streams")
    ap.add_argument("--any", action="store_true", help="overlap between any two dispatches")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, stream_id, queue_id from kernels order by start").fetchall()
    if a.last:
        rows = rows[-a.last:]
    by_stream = collections.Counter(r[3] for r in rows)
    main_stream = by_stream.most_common(1)[0][0]
    if len(by_stream) == 1 or a.any:
        # graph replays report every node on the launching stream: any two dispatches whose
        # intervals intersect ran concurrently (one stream would have serialised them)
        mains = [(s, e, n) for n, s, e, st, q in rows]
        side = [(s, e, n, st) for n, s, e, st, q in rows]
    else:
        mains = [(s, e, n) for n, s, e, st, q in rows if st == main_stream]
        side = [(s, e, n, st) for n, s, e, st, q in rows if st != main_stream]
    tot = collections.defaultdict(float)
    busy = collections.defaultdict(float)
    partners = collections.defaultdict(collections.Counter)
    j0 = 0
    for s, e, n, st in side:
        busy[n] += (e - s) / 1e3
        while j0 < len(mains) and mains[j0][0] + 200_000 < s:   # (intervals sorted by start)
            j0 += 1
        j = j0
        while j < len(mains) and mains[j][0] < e:
            ov = min(e, mains[j][1]) - max(s, mains[j][0])
            if ov > 0 and (mains[j][0], mains[j][1]) != (s, e):
                tot[n] += ov / 1e3
                partners[n][mains[j][2][:60]] += ov / 1e3
            j += 1
    lines = [f"# {a.title}", "", f"source: `{a.db}`; main stream {main_stream} "
             f"({by_stream[main_stream]} dispatches), side streams: "
             + ", ".join(f"{s} ({k})" for s, k in by_stream.items() if s != main_stream), "",
             "| side-stream kernel | busy us | overlapped with main-stream kernels us | overlapped with (top 3) |",
             "|---|---|---|---|"]
    for n in sorted(busy, key=lambda k: -busy[k]):
        top = "; ".join(f"`{p}` {v:.1f}" for p, v in partners[n].most_common(3))
        lines.append(f"| `{n[:70]}` | {busy[n]:.1f} | {tot[n]:.1f} | {top} |")
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        open(a.out, "w").write(text)


if __name__ == "__main__":
    main()
