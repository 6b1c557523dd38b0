#!/bin/bash
# round 6: column parts of the general-row kernels (option ryx_split: 0 one 8-wave part where it
# fits, 1 default, 2 parts of 2 waves, 3 parts of 1 wave) at a steady clock; parity of the split layouts
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
O=gpurun_out/r6/split.jsonl
: > $O
for c in w6 w4 w1 w5 w3 u2 u3 u1 h2; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --settle-ms 120 --reps 6 --block 8 \
    --arm auto: --arm s0:ryx_split=0 --arm s2:ryx_split=2 --arm s3:ryx_split=3 >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r6/split.jsonl"):
    d = json.loads(l)
    base = d["arms"]["auto"]["median_ms"]
    print(d["config"], d["frames"], " ".join("%s %.4f(%+.1f%%)" % (k, a["median_ms"], 100 * (a["median_ms"] / base - 1)) for k, a in d["arms"].items()),
          all(a["bit_exact_frame0"] for a in d["arms"].values()))
PY
