#!/bin/bash
# round 6: Lanczos-6 rows of 1..2:1 (ryg 16 taps, 10 pairs): 3 output columns per thread (default, spills a little) vs 2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
O=gpurun_out/r6/l6cpt.jsonl
: > $O
for s in lanczos,6,1920,1080,1366,768,256 lanczos,6,2560,1440,1920,1080,128 lanczos,5,1920,1080,1366,768,256; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --shape $s --settle-ms 120 --reps 6 --block 8 --arm auto: --arm c2:ryg_cpt=2 >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r6/l6cpt.jsonl"):
    d = json.loads(l)
    print(d["config"], d["frames"], " ".join("%s %s %.4f ms frac %.3f exact %s" % (k, a["kernel"], a["median_ms"], a["frac_median"], a["bit_exact_frame0"]) for k, a in d["arms"].items()))
PY
