#!/bin/bash
# A/B library variants on the C2 bench: scripts/ab.sh variantA.so variantB.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
for v in "$@"; do
  LIBIQO_AMD_LIB=$(pwd)/$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu ${BENCH_EXTRA} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "$v rep$rep $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["roofline"]["kernel_ms_per_launch"], d["parity"])')"
done
done
