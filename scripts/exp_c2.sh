#!/bin/bash
# C2 experiments: achievable bandwidth, store policy / memory-only variants, frames x bands, HBM traffic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
timeout -k 10 120 scripts/ubench/bw > "$OUT/bw.log" 2>&1 || { echo "bw failed"; tail -5 "$OUT/bw.log"; exit 1; }
cat "$OUT/bw.log"
REPS=2 bash scripts/ab2.sh "libiqo_amd/variants/base.so" "libiqo_amd/variants/ntst.so" \
  "libiqo_amd/variants/memonly.so|--no-verify" "libiqo_amd/variants/memonly_nt.so|--no-verify" \
  "libiqo_amd/variants/base.so|--frames 256" "libiqo_amd/variants/base.so|--frames 256 --bands 16" \
  "libiqo_amd/variants/base.so|--bands 8" "libiqo_amd/variants/ntst.so|--frames 256" || exit 1
cd /tmp || exit 1; export TMPDIR=/tmp
for fr in 128 256; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    LIBIQO_AMD_LIB=$ROOT/libiqo_amd/variants/base.so timeout -k 10 -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/pmc_${ctr}_$fr" -o run -- python3 "$ROOT/bench.py" --config c2 --frames $fr --steps 3 --warmup 1 --no-cpu --no-verify > "$OUT/pmc_${ctr}_$fr.log" 2>&1 || { echo "pmc $ctr $fr failed"; tail -5 "$OUT/pmc_${ctr}_$fr.log"; exit 1; }
    python3 - "$OUT/pmc_${ctr}_$fr/run_counter_collection.csv" $ctr $fr <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "iqo_amd" in r["Kernel_Name"]:
        tot[r["Dispatch_Id"]] += float(r["Counter_Value"])
v = sorted(tot.values())
print("%s frames=%s per-dispatch KiB: %s" % (sys.argv[2], sys.argv[3], ["%.0f" % x for x in v]))
PY
  done
done
