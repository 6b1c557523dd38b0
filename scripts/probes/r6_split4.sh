#!/bin/bash
# round 6: column parts of the exact-vertical-ratio kernel (ryx) at a steady clock
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
O=gpurun_out/r6/split4.jsonl
: > $O
for c in g5 h2 h6 h9 u1; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --settle-ms 120 --reps 6 --block 8 \
    --arm auto: --arm s0:ryx_split=0 --arm s2:ryx_split=2 --arm s3:ryx_split=3 >> $O || exit 1
done
for s in lanczos,3,2560,1440,640,360,256 lanczos,3,3840,2160,1920,960,128 lanczos,2,2560,1440,1138,640,256 \
         lanczos,3,1280,720,2880,1620,128 lanczos,6,2560,1440,1280,720,128 area,0,2560,1440,1138,640,256; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --shape $s --settle-ms 120 --reps 6 --block 8 \
    --arm auto: --arm s0:ryx_split=0 --arm s2:ryx_split=2 --arm s3:ryx_split=3 >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r6/split4.jsonl"):
    d = json.loads(l)
    base = d["arms"]["auto"]["median_ms"]
    print(d["config"], d["frames"], d["arms"]["auto"]["kernel"], " ".join("%s %.4f(%+.1f%%)" % (k, a["median_ms"], 100 * (a["median_ms"] / base - 1)) for k, a in d["arms"].items()),
          all(a["bit_exact_frame0"] for a in d["arms"].values()))
PY
