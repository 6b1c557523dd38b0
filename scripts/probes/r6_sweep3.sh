#!/bin/bash
# round 6: explicit band-count sweeps for the exact-ratio / streamer shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
O=gpurun_out/r6/sweep3.jsonl
: > $O
run() { c=$1; shift; a=(--arm auto:); for b in "$@"; do a+=(--arm b$b:bands=$b); done
  timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --settle-ms 120 --reps 6 --block 8 "${a[@]}" >> $O; }
run c1 5 8 12 15 20 || exit 1
run g1 8 16 24 45 90 || exit 1
run g2 27 54 108 216 || exit 1
run g4 8 16 30 60 90 || exit 1
run g5 10 20 40 80 || exit 1
run h2 10 20 45 90 || exit 1
run h4 27 54 108 216 || exit 1
run n2 3 6 12 24 || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/r6/sweep3.jsonl"):
    d = json.loads(l)
    base = d["arms"]["auto"]["median_ms"]
    print(d["config"], d["frames"], " ".join("%s %.4f(%+.1f%%)" % (k, a["median_ms"], 100 * (a["median_ms"] / base - 1)) for k, a in d["arms"].items()),
          all(a["bit_exact_frame0"] for a in d["arms"].values()))
PY
