#!/bin/bash
# round 6: C2 per-launch fixed cost (frames sweep) and 256-frame band / tail options, steady clock
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/r6_fixed.jsonl
: > $O
for f in 32 64 128 256 512 1024; do
  timeout -k 10 120 python scripts/probes/steady_ab.py --config c2 --frames $f --settle-ms 150 --reps 6 --block 8 --arm base: >> $O || exit 1
done
timeout -k 10 200 python scripts/probes/steady_ab.py --config c2 --frames 256 --settle-ms 150 --reps 8 --block 8 \
  --arm base: --arm b96:bands=96 --arm b88:bands=88 --arm notail:tail=-1 --arm tail4:tail=270 --arm tail6:tail=180 >> $O || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/r6_fixed.jsonl"):
    d = json.loads(l)
    for k, a in d["arms"].items():
        print(d["frames"], k, a["median_ms"], a["min_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
