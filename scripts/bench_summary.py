"""Print ms_per_step of bench.py JSON lines from log files, grouped by tag (file name minus _<run>.log).

    python scripts/bench_summary.py gpurun_out/r3ab/*.log
"""
import collections
import json
import os
import re
import sys


def main(paths):
    groups = collections.OrderedDict()
    for p in sorted(paths):
        tag = re.sub(r"_\d+$", "", os.path.basename(p)[:-4])
        ms = None
        try:
            for line in open(p):
                if line.startswith("{"):
                    ms = json.loads(line).get("ms_per_step")
        except OSError:
            pass
        if ms is not None:
            groups.setdefault(tag, []).append(ms)
    for tag, v in groups.items():
        print(f"{tag:28s} " + " ".join(f"{x:.4f}" for x in v))


if __name__ == "__main__":
    main(sys.argv[1:])
