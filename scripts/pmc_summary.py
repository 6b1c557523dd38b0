"""Per-dispatch averages of PMC counters for the hot kernel: pmc_summary.py OUTDIR TAG NPASSES"""
import collections
import csv
import sys

out, tag, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
tot, cnt = collections.defaultdict(float), collections.defaultdict(set)
for i in range(1, n + 1):
    with open("%s/pmc_%s%d/run_counter_collection.csv" % (out, tag, i)) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if "iqo_amd" not in name:
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(tot):
    print("%-26s %16.0f  (per dispatch, %d dispatches)" % (k, tot[k] / len(cnt[k]), len(cnt[k])))
