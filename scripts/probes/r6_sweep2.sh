#!/bin/bash
# round 6: band sweeps around the auto choice for the exact-ratio / streamer shapes; two-rank bench GPU test
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
true

O=gpurun_out/r6/sweep2.jsonl
: > $O
timeout -k 10 200 python scripts/probes/band_sweep.py c1 "st2:stack=2" "notail:tail=-1" >> $O || exit 1
for c in g1 g2 g4 g5 h2 h4 n1 n2; do
  timeout -k 10 200 python scripts/probes/band_sweep.py $c >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r6/sweep2.jsonl"):
    d = json.loads(l)
    base = d["arms"]["auto"]["median_ms"]
    print(d["config"], d["frames"], d["tag"], " ".join("%s %.4f(%+.1f%%)" % (k, a["median_ms"], 100 * (a["median_ms"] / base - 1)) for k, a in d["arms"].items()),
          all(a["bit_exact_frame0"] for a in d["arms"].values()))
PY
