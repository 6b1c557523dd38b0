#!/bin/bash
# symmetric streamer: prefetch x debug flags (3 = compute only) x bands on C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for pd in 1 2 3; do for f in 0 3; do for b in 0 6 8 12; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu --no-verify --prefetch $pd --debug-flags $f --bands $b ${BENCH_EXTRA} > gpurun_out/exp.log 2>&1 || { tail -5 gpurun_out/exp.log; exit 1; }
  echo "pd=$pd flags=$f bands=$b $(tail -1 gpurun_out/exp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["roofline"]["kernel_ms_per_launch"])')"
done; done; done
