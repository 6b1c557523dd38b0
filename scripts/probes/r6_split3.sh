#!/bin/bash
# round 6: the general-row kernels' one-wave column parts (new default) vs the previous rule (ryx_split=4);
# GPU suite first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/gpu_tests_split3.txt 2>&1 || { tail -30 gpurun_out/r6/gpu_tests_split3.txt; exit 1; }
tail -1 gpurun_out/r6/gpu_tests_split3.txt
O=gpurun_out/r6/split3.jsonl
: > $O
for c in w1 w3 w4 w5 w6 w7 u2 u3; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --settle-ms 120 --reps 6 --block 8 --arm new: --arm old:ryx_split=4 >> $O || exit 1
done
for s in lanczos,3,3840,2160,1600,900,128 lanczos,3,2560,1440,1024,576,256 lanczos,2,3840,2160,1366,768,128 \
         lanczos,3,1920,1080,768,432,256 lanczos,3,1920,1080,1600,900,256 lanczos,3,2560,1440,1920,1080,128 \
         lanczos,2,1920,1080,1366,768,256 lanczos,2,3840,2160,1024,576,128 lanczos,3,1366,768,2560,1440,128 \
         lanczos,4,1920,1080,1366,768,256 lanczos,4,3840,2160,2560,1440,64 lanczos,2,1600,900,1920,1080,256; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --shape $s --settle-ms 120 --reps 6 --block 8 --arm new: --arm old:ryx_split=4 >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r6/split3.jsonl"):
    d = json.loads(l)
    n, o = d["arms"]["new"], d["arms"]["old"]
    print("%-34s %4d %-6s new %.4f old %.4f (%+.1f%%) frac %.3f -> %.3f %s" % (d["config"], d["frames"], n["kernel"], n["median_ms"], o["median_ms"],
          100 * (n["median_ms"] / o["median_ms"] - 1), o["frac_median"], n["frac_median"], n["bit_exact_frame0"] and o["bit_exact_frame0"]))
PY
