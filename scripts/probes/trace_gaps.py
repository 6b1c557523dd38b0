#!/usr/bin/env python3
"""Per-grid-size dispatch duration and inter-dispatch gap of the dominant kernel in a rocprofv3
kernel-trace CSV (GPU-box tooling): separates a kernel's per-launch fixed cost into the part inside
the dispatch (ramp / tail) and the gap between back-to-back dispatches.

usage: trace_gaps.py KERNEL_TRACE_CSV [--skip N]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    skip = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[2] == "--skip" else 40
    rows = list(csv.DictReader(open(path)))
    tot = collections.Counter()
    for r in rows:
        tot[r["Kernel_Name"]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    for name, _ in tot.most_common(3):
        seq = [r for r in rows if r["Kernel_Name"] == name]
        groups = collections.OrderedDict()
        for i, r in enumerate(seq):
            g = int(r.get("Grid_Size", 0) or 0) or int(r.get("Grid_Size_X", 0) or 0)
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            gap = None
            if i + 1 < len(seq):
                gap = (int(seq[i + 1]["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1e3
            groups.setdefault(g, []).append((dur, gap))
        print("# kernel:", name.split("(")[0][:90])
        for g, v in groups.items():
            v2 = v[skip:] if len(v) > skip + 8 else v
            d = sorted(x[0] for x in v2)
            gaps = sorted(x[1] for x in v2 if x[1] is not None and x[1] < 50)
            print("grid %9d: %4d dispatches (%d used)  dur median %.2f us  min %.2f  gap median %s us"
                  % (g, len(v), len(v2), d[len(d) // 2], d[0],
                     "%.2f" % gaps[len(gaps) // 2] if gaps else "-"))


if __name__ == "__main__":
    main()
