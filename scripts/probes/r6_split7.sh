#!/bin/bash
# round 6: ryx one-wave parts for Lanczos rows whose parts are < 3/4 busy (new default) vs the previous
# rule (ryx_split=4); ryx parity first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ryx or ratio or random or golden or band" > gpurun_out/r6/gpu_tests_split7.txt 2>&1 || { tail -30 gpurun_out/r6/gpu_tests_split7.txt; exit 1; }
tail -1 gpurun_out/r6/gpu_tests_split7.txt
O=gpurun_out/r6/split7.jsonl
: > $O
for c in g5 h2 h6 u1; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --settle-ms 120 --reps 6 --block 8 --arm new: --arm old:ryx_split=4 >> $O || exit 1
done
for s in lanczos,3,2560,1440,640,360,256 lanczos,2,2560,1440,1138,640,256 lanczos,6,2560,1440,1280,720,128 \
         lanczos,3,1280,720,2880,1620,128 lanczos,3,2560,1440,1280,720,128 lanczos,3,3840,2160,1920,960,128 lanczos,4,2560,1440,640,360,256; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --shape $s --settle-ms 120 --reps 6 --block 8 --arm new: --arm old:ryx_split=4 >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r6/split7.jsonl"):
    d = json.loads(l)
    n, o = d["arms"]["new"], d["arms"]["old"]
    print("%-34s %4d %-14s new %.4f old %.4f (%+.1f%%) frac %.3f -> %.3f %s" % (d["config"], d["frames"], n["kernel"], n["median_ms"], o["median_ms"],
          100 * (n["median_ms"] / o["median_ms"] - 1), o["frac_median"], n["frac_median"], n["bit_exact_frame0"] and o["bit_exact_frame0"]))
PY
bash scripts/probes/r6_split6.sh
