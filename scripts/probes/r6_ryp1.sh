#!/bin/bash
# round 6: ryp (downscale rows by window position) parity + A/B vs ryg
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ryg or random or golden" > gpurun_out/r6/gpu_tests_ryp1.txt 2>&1 || { tail -40 gpurun_out/r6/gpu_tests_ryp1.txt; exit 1; }
tail -2 gpurun_out/r6/gpu_tests_ryp1.txt
O=gpurun_out/r6/ryp1.jsonl
: > $O
for c in w1 w2 w3 w4 w5 w6 w7; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --settle-ms 120 --reps 8 --block 8 --arm ryp: --arm ryg:ryp=0 >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r6/ryp1.jsonl"):
    d = json.loads(l)
    for k, a in d["arms"].items():
        print(d["config"], d["frames"], k, a["kernel"], a["median_ms"], a["min_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
