#!/bin/bash
# round 6: C4 (linear_up2) strip width / band A/B at a steady clock, and C2 per-launch fixed cost
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
O=gpurun_out/r6/c4lanes.jsonl
: > $O
timeout -k 10 200 python scripts/probes/steady_ab.py --config c4 --frames 256 --settle-ms 150 --reps 8 --block 8 \
  --arm base: --arm l48:lanes=48 --arm l40:lanes=40 --arm l56:lanes=56 --arm l32:lanes=32 --arm l62:lanes=62 >> $O || exit 1
timeout -k 10 200 python scripts/probes/steady_ab.py --config c4 --frames 256 --settle-ms 150 --reps 8 --block 8 \
  --arm base: --arm l48:lanes=48 --arm l48b24:lanes=48,bands=24 --arm l48b96:lanes=48,bands=96 --arm b24:bands=24 --arm b96:bands=96 >> $O || exit 1
O2=gpurun_out/r6/c2frames.jsonl
: > $O2
for f in 64 256 1024; do
  timeout -k 10 120 python scripts/probes/steady_ab.py --config c2 --frames $f --settle-ms 150 --reps 6 --block 8 --arm base: >> $O2 || exit 1
done
timeout -k 10 200 python scripts/probes/steady_ab.py --config c2 --frames 256 --settle-ms 150 --reps 8 --block 8 \
  --arm base: --arm b96:bands=96 --arm notail:tail=-1 --arm tail4:tail=270 --arm tail6:tail=180 >> $O2 || exit 1
python - <<'PY'
import json
for f in ("gpurun_out/r6/c4lanes.jsonl", "gpurun_out/r6/c2frames.jsonl"):
    for l in open(f):
        d = json.loads(l)
        for k, a in d["arms"].items():
            print(d["config"], d["frames"], k, a["median_ms"], a["min_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
