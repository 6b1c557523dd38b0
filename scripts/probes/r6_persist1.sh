#!/bin/bash
# round 6: queued resident C2 streamer -- parity, steady A/B against the one-shot grid, timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "1024 or batch or c2 or lanczos3 or golden or padded or relaunch" > gpurun_out/r6/gpu_tests_persist1.txt 2>&1 || { tail -40 gpurun_out/r6/gpu_tests_persist1.txt; exit 1; }
tail -3 gpurun_out/r6/gpu_tests_persist1.txt
O=gpurun_out/r6/persist1.jsonl
: > $O
for f in 256 1024; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --config c2 --frames $f --settle-ms 150 --reps 8 --block 6 \
    --arm persist: --arm oneshot:persist=-1 --arm pool2:persist=2 --arm pool8:persist=8 >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r6/persist1.jsonl"):
    d = json.loads(l)
    for k, a in d["arms"].items():
        print(d["config"], d["frames"], k, a["kernel"], a["median_ms"], a["min_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
export LIBIQO_AMD_LIB=$GRAFT_REPO_ROOT/libiqo_amd/variants/trace.so
for f in 256 1024; do
  timeout -k 10 120 python scripts/probes/wg_trace.py --frames $f --dump gpurun_out/r6/ptrace_$f.npy >> gpurun_out/r6/ptrace.jsonl || exit 1
done
cat gpurun_out/r6/ptrace.jsonl
