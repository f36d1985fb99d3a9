"""Host-side launch cost of graph replays from a rocprofv3 --sys-trace database (rocpd SQLite):
HIP API durations by name, and for each hipGraphLaunch the time from the call's start to the
first kernel that starts after it (how long the GPU waits for the host).

    python scripts/api_gaps.py <run_results.db> > summary.txt
"""
import collections
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    objs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    print("tables/views:", ", ".join(o for o in objs if not o.startswith("rocpd_info")))
    api_tab = next((t for t in ("regions", "apis", "api", "region") if t in objs), None)
    if api_tab is None:
        print("no API view found")
        return
    cols = [r[1] for r in c.execute(f"pragma table_info({api_tab})")]
    print(f"{api_tab} columns:", ", ".join(cols))
    name_col = "name" if "name" in cols else cols[0]
    rows = list(c.execute(f"select {name_col}, start, end from {api_tab} order by start"))
    by = collections.defaultdict(list)
    for n, s, e in rows:
        by[n].append((e - s) / 1e3)
    print("\nHIP API calls (count, mean us, max us), top 25 by total time:")
    for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:25]:
        print(f"  {n[:60]:60s} {len(v):7d} {sum(v) / len(v):9.2f} {max(v):9.2f}")
    kern = list(c.execute("select start, end, name from kernels order by start"))
    ks = [k[0] for k in kern]
    import bisect
    launches = [(s, e) for n, s, e in rows if "GraphLaunch" in n]
    print(f"\nhipGraphLaunch calls: {len(launches)}")
    for s, e in launches[-12:]:
        i = bisect.bisect_left(ks, s)
        first = kern[i] if i < len(kern) else None
        prev_end = max((k[1] for k in kern[:i]), default=0)
        print(f"  call {(e - s) / 1e3:8.2f} us; first kernel starts {(first[0] - s) / 1e3 if first else -1:8.2f} us "
              f"after the call ({first[2][:30] if first else '-'}); GPU idle before it "
              f"{(first[0] - prev_end) / 1e3 if first else -1:8.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])
