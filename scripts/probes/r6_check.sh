#!/bin/bash
# round 6: GPU suite, smoke and default bench on the current tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r6/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r6/gpu_tests.txt; exit 1; }
tail -3 gpurun_out/r6/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/smoke.txt 2>&1 || exit 1
cat gpurun_out/r6/smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/r6/bench_default.json 2> gpurun_out/r6/bench_default.err || { tail -20 gpurun_out/r6/bench_default.err; exit 1; }
cat gpurun_out/r6/bench_default.json
