#!/bin/bash
# round 6: column parts (ryx_split 2 = parts of 2 waves, 3 = parts of 1 wave) on more general-row shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
O=gpurun_out/r6/split2.jsonl
: > $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ryg or ryu or random" > gpurun_out/r6/gpu_tests_split2.txt 2>&1 || { tail -30 gpurun_out/r6/gpu_tests_split2.txt; exit 1; }
tail -1 gpurun_out/r6/gpu_tests_split2.txt
for c in u2 u3; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --settle-ms 120 --reps 6 --block 8 --arm auto: --arm old18:bands=18 >> $O || exit 1
done
for s in lanczos,3,3840,2160,1600,900,128 lanczos,3,2560,1440,1024,576,256 lanczos,2,3840,2160,1366,768,128 \
         lanczos,3,1920,1080,768,432,256 lanczos,3,3840,2160,1366,768,128 lanczos,4,3840,2160,1366,768,128 \
         lanczos,3,1920,1080,1600,900,256 lanczos,3,2560,1440,1920,1080,128 lanczos,2,1920,1080,1366,768,256 \
         lanczos,2,3840,2160,1024,576,128 lanczos,3,1366,768,2560,1440,128 lanczos,3,1024,576,1920,1080,256 \
         lanczos,3,1366,768,1920,1080,256 lanczos,2,1366,768,1920,1080,256; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --shape $s --settle-ms 120 --reps 6 --block 8 \
    --arm auto: --arm s2:ryx_split=2 --arm s3:ryx_split=3 >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r6/split2.jsonl"):
    d = json.loads(l)
    base = d["arms"]["auto"]["median_ms"]
    print(d["config"], d["frames"], d["arms"]["auto"]["kernel"], " ".join("%s %.4f(%+.1f%%)" % (k, a["median_ms"], 100 * (a["median_ms"] / base - 1)) for k, a in d["arms"].items()),
          all(a["bit_exact_frame0"] for a in d["arms"].values()))
PY
