#!/bin/bash
# round 6: up to 32 column parts (one-wave parts of 4K rows): W4 / W6 and 4K shapes, new vs the 2-wave
# parts (ryx_split=2) and the rule before one-wave parts (ryx_split=4); ryg / ryx parity first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ryg or ryu or ryx or random or band" > gpurun_out/r6/gpu_tests_split5.txt 2>&1 || { tail -30 gpurun_out/r6/gpu_tests_split5.txt; exit 1; }
tail -1 gpurun_out/r6/gpu_tests_split5.txt
O=gpurun_out/r6/split5.jsonl
: > $O
for c in w4 w6 w5 w1; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --settle-ms 120 --reps 6 --block 8 --arm new: --arm s2:ryx_split=2 --arm old:ryx_split=4 >> $O || exit 1
done
for s in lanczos,3,3840,2160,1600,900,128 lanczos,4,3840,2160,1366,768,128 lanczos,3,3840,2160,1920,1200,64 lanczos,2,3840,2160,1366,768,128; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --shape $s --settle-ms 120 --reps 6 --block 8 --arm new: --arm s2:ryx_split=2 --arm old:ryx_split=4 >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r6/split5.jsonl"):
    d = json.loads(l)
    base = d["arms"]["old"]["median_ms"]
    print("%-34s %4d %-6s" % (d["config"], d["frames"], d["arms"]["new"]["kernel"]), " ".join("%s %.4f(%+.1f%%) %.3f" % (k, a["median_ms"], 100 * (a["median_ms"] / base - 1), a["frac_median"]) for k, a in d["arms"].items()),
          all(a["bit_exact_frame0"] for a in d["arms"].values()))
PY
