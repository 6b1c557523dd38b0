#!/bin/bash
# round 6: steady bench line per config (the DESIGN table)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
BENCH_EXTRA="--warmup 100 --steps 50" bash scripts/gpu_ci.sh benchlines || exit 1
mkdir -p gpurun_out/r6 && cp gpurun_out/bench_lines.jsonl gpurun_out/r6/bench_lines.jsonl
