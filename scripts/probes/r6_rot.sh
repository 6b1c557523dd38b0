#!/bin/bash
# round 6: ryg per-lane LDS read rotation vs none (option ryg_rot=0); ryg parity
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ryg or random or golden" > gpurun_out/r6/gpu_tests_rot.txt 2>&1 || { tail -30 gpurun_out/r6/gpu_tests_rot.txt; exit 1; }
tail -2 gpurun_out/r6/gpu_tests_rot.txt
O=gpurun_out/r6/rot.jsonl
: > $O
for c in w4 w6 w5 w1 w3; do
  timeout -k 10 120 python scripts/probes/steady_ab.py --config $c --settle-ms 100 --reps 8 --block 8 --arm rot: --arm norot:ryg_rot=0 >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r6/rot.jsonl"):
    d = json.loads(l)
    for k, a in d["arms"].items():
        print(d["config"], d["frames"], k, a["median_ms"], a["min_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
