#!/bin/bash
# round 6: ryu (upscale rows by window position) parity + A/B vs ryg NL=1; C4 band/lane sweep; C2 lanes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "ryg or random or golden" > gpurun_out/r6/gpu_tests_ryu1.txt 2>&1 || { tail -40 gpurun_out/r6/gpu_tests_ryu1.txt; exit 1; }
tail -3 gpurun_out/r6/gpu_tests_ryu1.txt
O=gpurun_out/r6/ryu1.jsonl
: > $O
for c in u2 u3; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --frames 256 --settle-ms 150 --reps 8 --block 8 \
    --arm ryu: --arm ryg:ryu=0 >> $O || exit 1
done
timeout -k 10 300 python scripts/probes/steady_ab.py --config c4 --frames 256 --settle-ms 150 --reps 8 --block 8 \
  --arm l48b216:lanes=48,bands=216 --arm l48b180:lanes=48,bands=180 --arm l48b270:lanes=48,bands=270 \
  --arm l48b360:lanes=48,bands=360 --arm l48b432:lanes=48,bands=432 --arm l40b216:lanes=40,bands=216 \
  --arm l40b270:lanes=40,bands=270 --arm l60b270:lanes=60,bands=270 --arm l32b270:lanes=32,bands=270 >> $O || exit 1
timeout -k 10 200 python scripts/probes/steady_ab.py --config c2 --frames 256 --settle-ms 150 --reps 8 --block 8 \
  --arm base: --arm l48:lanes=48 --arm l40:lanes=40 >> $O || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/r6/ryu1.jsonl"):
    d = json.loads(l)
    for k, a in d["arms"].items():
        print(d["config"], d["frames"], k, a["kernel"], a["median_ms"], a["min_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
