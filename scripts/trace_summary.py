#!/usr/bin/env python3
"""Per-dispatch summary of a rocprofv3 --kernel-trace CSV for the bench's dominant kernel.

usage: trace_summary.py KERNEL_TRACE_CSV BENCH_LINE_JSON [--steps 20 --warmup 5]

Groups the dispatches of the kernel that takes most of the time by grid size (the headline batch
and bench.py's batch_alt), prints each group's per-dispatch milliseconds in launch order, and for
the headline batch the mean of the timed launches next to the bench line's own HIP-event figure
(the two must agree: ROUND contract, roofline.achieved)."""
import argparse
import collections
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("line")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--kernel", default="", help="substring of the kernel to summarise (default: the one taking most time)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    tot = collections.Counter()
    for r in rows:
        tot[r["Kernel_Name"]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    top = tot.most_common(1)[0][0]
    if a.kernel:  # (the default bench also launches the C3 / C4 secondary lines and probes)
        top = max((k for k in tot if a.kernel in k), key=lambda k: tot[k])
    groups = collections.OrderedDict()
    for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
        if r["Kernel_Name"] != top:
            continue
        g = int(r.get("Grid_Size", 0) or 0) or int(r.get("Grid_Size_X", 0) or 0)
        groups.setdefault(g, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    line = json.loads(open(a.line).read().strip().splitlines()[-1])
    print("# kernel:", top.split("<")[0].replace("void ", ""))
    for i, (g, ms) in enumerate(groups.items()):
        s = sorted(ms)
        print("\n## grid %d: %d dispatches, mean %.4f, median %.4f, min %.4f ms"
              % (g, len(ms), sum(ms) / len(ms), s[len(s) // 2], s[0]))
        if i == 0 and len(ms) >= a.warmup + a.steps:
            t = ms[a.warmup:a.warmup + a.steps]
            m = sum(t) / len(t)
            r = line["roofline"]
            print("## timed launches %d..%d: mean %.4f ms; the bench line's HIP-event figure: %.4f ms, frac %.4f"
                  % (a.warmup, a.warmup + a.steps - 1, m, r["kernel_ms_per_launch"], r["frac"]))
        for k in range(0, len(ms), 16):
            print("  " + " ".join("%.3f" % v for v in ms[k:k + 16]))


if __name__ == "__main__":
    main()
