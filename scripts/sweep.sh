#!/bin/bash
# Sweep bench argument sets: scripts/sweep.sh "--prefetch 1" "--prefetch 2 --bands 8" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for a in "$@"; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu $a > gpurun_out/sweep.log 2>&1 || { echo "FAILED: $a"; tail -5 gpurun_out/sweep.log; exit 1; }
  echo "[$a] $(tail -1 gpurun_out/sweep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["roofline"]["kernel_ms_per_launch"], d["parity"][:9])')"
done
