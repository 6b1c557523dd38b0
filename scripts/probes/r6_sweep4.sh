#!/bin/bash
# round 6: band-count sweeps for the general-row kernels (ryu U2/U3, ryx U1/H6/H9, ryg W1/W4)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
O=gpurun_out/r6/sweep4.jsonl
: > $O
run() { c=$1; shift; a=(--arm auto:); for b in "$@"; do a+=(--arm b$b:bands=$b); done
  timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --settle-ms 120 --reps 6 --block 8 "${a[@]}" >> $O; }
run u2 6 9 12 27 36 54 || exit 1
run u3 6 9 12 27 36 54 || exit 1
run u1 4 8 15 30 60 || exit 1
run h6 5 10 20 40 || exit 1
run h9 5 10 20 40 || exit 1
run w1 6 12 24 36 || exit 1
run w4 3 6 12 24 || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/r6/sweep4.jsonl"):
    d = json.loads(l)
    base = d["arms"]["auto"]["median_ms"]
    print(d["config"], d["frames"], " ".join("%s %.4f(%+.1f%%)" % (k, a["median_ms"], 100 * (a["median_ms"] / base - 1)) for k, a in d["arms"].items()),
          all(a["bit_exact_frame0"] for a in d["arms"].values()))
PY
