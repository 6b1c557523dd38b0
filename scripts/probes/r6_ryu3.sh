#!/bin/bash
# round 6: ryu with the next position's scalar loads pinned before the barrier
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ryg" > gpurun_out/r6/gpu_tests_ryu3.txt 2>&1 || { tail -40 gpurun_out/r6/gpu_tests_ryu3.txt; exit 1; }
tail -2 gpurun_out/r6/gpu_tests_ryu3.txt
O=gpurun_out/r6/ryu3.jsonl
: > $O
for c in u2 u3; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --frames 256 --settle-ms 150 --reps 8 --block 8 \
    --arm run: --arm ryg:ryu=0 >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r6/ryu3.jsonl"):
    d = json.loads(l)
    for k, a in d["arms"].items():
        print(d["config"], d["frames"], k, a["kernel"], a["median_ms"], a["min_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
