#!/bin/bash
# Sweep bench argument sets on one config, REPS interleaved repetitions:
#   CFG=c4 REPS=2 scripts/sweep_cfg.sh "" "--option lin_prefetch=8" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-1}); do
for a in "$@"; do
  timeout -k 10 120 python bench.py --config ${CFG:-c2} --steps 20 --warmup 3 --no-cpu $a > gpurun_out/sweep.log 2>&1 || { echo "FAILED: $a"; tail -5 gpurun_out/sweep.log; exit 1; }
  echo "${CFG:-c2} [$a] $(tail -1 gpurun_out/sweep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["roofline"]["kernel_ms_per_launch"], d["parity"][:9])')"
done
done
