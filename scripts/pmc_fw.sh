#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per dispatch of one bench command (separate passes):
#   TAG=x scripts/pmc_fw.sh --config c2 --frames 128 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd /tmp || exit 1; export TMPDIR=/tmp
TAG=${TAG:-fw}
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/pmc_${TAG}_$ctr" -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-verify "$@" > "$OUT/pmc_${TAG}_$ctr.log" 2>&1 || { echo "pmc $ctr failed"; tail -5 "$OUT/pmc_${TAG}_$ctr.log"; exit 1; }
  python3 - "$OUT/pmc_${TAG}_$ctr/run_counter_collection.csv" $ctr "$TAG" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "iqo_amd" in r["Kernel_Name"]:
        tot[r["Dispatch_Id"]] += float(r["Counter_Value"])
v = sorted(tot.values())
print("%s %s per-dispatch KiB: %s" % (sys.argv[3], sys.argv[2], ["%.0f" % x for x in v]))
PY
done
