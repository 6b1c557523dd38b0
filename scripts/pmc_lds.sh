#!/bin/bash
# LDS counters for bench configs (one rocprofv3 --pmc pass each, kernel-trace only beside it).
#   CFGS="g5 h2" scripts/pmc_lds.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd /tmp || exit 1; export TMPDIR=/tmp
for c in ${CFGS:-g5}; do
  timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CU_CYCLES --kernel-trace --output-format csv -d "$OUT/pmc_lds_$c" -o run -- python3 "$ROOT/bench.py" --config $c --steps 2 --warmup 1 --no-cpu --no-verify --no-probe --alt-frames 0 > "$OUT/pmc_lds_$c.log" 2>&1 || { echo "lds pass $c failed"; tail -5 "$OUT/pmc_lds_$c.log"; exit 1; }
  python3 - "$OUT/pmc_lds_$c" "$c" <<'PY'
import csv, glob, sys, collections
d, c = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for fn in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(fn)):
        if "iqo_amd" not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (disp, name), v in per.items():
        acc[name].append(v)
for name in sorted(acc):
    v = acc[name]
    print("%s %-24s %14.0f (mean of %d dispatches)" % (c, name, sum(v) / len(v), len(v)))
PY
done
