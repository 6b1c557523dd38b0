#!/bin/bash
# Sweep bench argument sets, REPS interleaved repetitions (box-to-box variance is ~5%, so compare
# within one call):  REPS=2 scripts/sweep.sh "--prefetch 1" "--prefetch 2 --bands 8" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-1}); do
for a in "$@"; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu $a > gpurun_out/sweep.log 2>&1 || { echo "FAILED: $a"; tail -5 gpurun_out/sweep.log; exit 1; }
  echo "[$a] $(tail -1 gpurun_out/sweep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["roofline"]["kernel_ms_per_launch"], d["parity"][:9])')"
done
done
