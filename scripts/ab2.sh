#!/bin/bash
# A/B library variants with per-variant bench args, interleaved:  scripts/ab2.sh "lib.so|--args" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
for spec in "$@"; do
  v=${spec%%|*}; args=${spec#*|}; [ "$args" = "$spec" ] && args=""
  LIBIQO_AMD_LIB=$(pwd)/$v timeout -k 10 120 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu ${BENCH_EXTRA} $args > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "$v [$args] rep$rep $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["roofline"]["kernel_ms_per_launch"], d["parity"][:9])')"
done
done
