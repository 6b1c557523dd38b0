#!/bin/bash
# round 6: column parts of the general-row kernels for Area and Linear rows (ryx_split 2 / 3 vs auto)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
O=gpurun_out/r6/split6.jsonl
: > $O
for c in w2 w7; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --settle-ms 120 --reps 6 --block 8 \
    --arm auto: --arm s2:ryx_split=2 --arm s3:ryx_split=3 >> $O || exit 1
done
for s in area,0,2560,1440,1920,1080,128 area,0,2560,1440,1024,576,256 area,0,1920,1080,1600,900,256 \
         linear,0,2560,1440,1920,1080,128 linear,0,1920,1080,1600,900,256 linear,0,1920,1080,1024,576,256; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --shape $s --settle-ms 120 --reps 6 --block 8 \
    --arm auto: --arm s2:ryx_split=2 --arm s3:ryx_split=3 >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r6/split6.jsonl"):
    d = json.loads(l)
    base = d["arms"]["auto"]["median_ms"]
    print(d["config"], d["frames"], d["arms"]["auto"]["kernel"], " ".join("%s %.4f(%+.1f%%)" % (k, a["median_ms"], 100 * (a["median_ms"] / base - 1)) for k, a in d["arms"].items()),
          all(a["bit_exact_frame0"] for a in d["arms"].values()))
PY
