#!/bin/bash
# interleaved A/B of bench option sets: scripts/probes/ab_opts.sh "args" "args" ...   (REPS, STEPS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
for args in "$@"; do
  timeout -k 10 120 python bench.py --steps ${STEPS:-30} --warmup 3 --no-cpu --no-probe ${BENCH_EXTRA} $args > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "[$args] rep$rep $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel_ms_per_launch"], round(r["kernel_ms_per_launch"]/d["config"]["frames_per_gpu"],6), r["frac"], d["parity"][:9])')"
done
done
