#!/bin/bash
# round 6: the new band rules (auto) vs the old choices (explicit), plus parity of the affected kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "up2 or d32 or d31 or golden or random or exact" > gpurun_out/r6/gpu_tests_bands4.txt 2>&1 || { tail -30 gpurun_out/r6/gpu_tests_bands4.txt; exit 1; }
tail -2 gpurun_out/r6/gpu_tests_bands4.txt
O=gpurun_out/r6/bands4.jsonl
: > $O
timeout -k 10 200 python scripts/probes/steady_ab.py --config g4 --settle-ms 120 --reps 6 --block 8 --arm new: --arm old:bands=8 >> $O || exit 1
timeout -k 10 200 python scripts/probes/steady_ab.py --config g1 --settle-ms 120 --reps 6 --block 8 --arm new: --arm old:bands=24 >> $O || exit 1
timeout -k 10 200 python scripts/probes/steady_ab.py --config h4 --settle-ms 120 --reps 6 --block 8 --arm new: --arm old:bands=120 >> $O || exit 1
timeout -k 10 200 python scripts/probes/steady_ab.py --config g2 --settle-ms 120 --reps 6 --block 8 --arm new: --arm old:bands=180 >> $O || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/r6/bands4.jsonl"):
    d = json.loads(l)
    for k, a in d["arms"].items():
        print(d["config"], d["frames"], k, a["kernel"], a["median_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
