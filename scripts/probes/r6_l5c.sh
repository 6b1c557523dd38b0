#!/bin/bash
# round 6: Lanczos-5 / -6 rows of 1..2:1 on ryg (new instantiations) vs the kernel
# they had (option ryg=0); ryg parity first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ryg or random" > gpurun_out/r6/gpu_tests_l5c.txt 2>&1 || { tail -30 gpurun_out/r6/gpu_tests_l5c.txt; exit 1; }
tail -1 gpurun_out/r6/gpu_tests_l5c.txt
O=gpurun_out/r6/l5c.jsonl
: > $O
for s in lanczos,5,3840,2160,1366,768,128 lanczos,5,2560,1440,1024,576,256; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --shape $s --settle-ms 120 --reps 4 --block 4 --arm ryg: --arm before:ryg=0 >> $O || exit 1
done
for c in w4; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --settle-ms 120 --reps 6 --block 8 --arm now: >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r6/l5c.jsonl"):
    d = json.loads(l)
    print(d["config"], d["frames"], " ".join("%s %s %.4f ms frac %.3f exact %s" % (k, a["kernel"], a["median_ms"], a["frac_median"], a["bit_exact_frame0"]) for k, a in d["arms"].items()))
PY
