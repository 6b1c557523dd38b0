#!/bin/bash
# UTCL1 translation counters per C2 dispatch, 3 rotated batches (separate --pmc passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; cd /tmp || exit 1; export TMPDIR=/tmp
i=0
for set in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum" "TCP_UTCL1_PERMISSION_MISS_sum TCP_UTCL1_REQUEST_sum" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/pmc_tlb$i" -o run -- python3 "$ROOT/scripts/probes/tlb_probe.py" > "$OUT/pmc_tlb$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/pmc_tlb$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for i in (1, 2, 3):
    rows = collections.defaultdict(dict)
    durs = {}
    for fn in glob.glob(out + "/pmc_tlb%d/**/*counter_collection.csv" % i, recursive=True):
        for r in csv.DictReader(open(fn)):
            if "lanczos_symb" not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            rows[d][r["Counter_Name"]] = rows[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(rows)
    for k, d in enumerate(ids):
        print("pass %d launch %2d batch %d %s" % (i, k, k % 3, " ".join("%s=%.4g" % (n, v) for n, v in sorted(rows[d].items()))))
PY
