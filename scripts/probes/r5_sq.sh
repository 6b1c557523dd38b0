#!/bin/bash
# SQ / LDS counters of the ryx (Lanczos-6 / -9 2:1) and ryg (1080p -> 1366x768) kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
for c in w1 h6 h9; do
  CFG=$c TAG=sq_$c bash scripts/pmc_sq.sh > "$OUT/sq_$c.txt" 2>&1 || { echo "sq $c failed"; tail -20 "$OUT/sq_$c.txt"; exit 1; }
done
CFGS="w1 w3 h9" bash scripts/pmc_lds.sh > "$OUT/lds_w1.txt" 2>&1 || { echo "lds failed"; tail -20 "$OUT/lds_w1.txt"; exit 1; }
cat "$OUT"/sq_w1.txt "$OUT"/lds_w1.txt
