#!/bin/bash
# round 6: ryu with up to 3 rows per window position; U1 (4:9 rows) on ryu (variant) vs ryx
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ryg or random" > gpurun_out/r6/gpu_tests_ryu4.txt 2>&1 || { tail -40 gpurun_out/r6/gpu_tests_ryu4.txt; exit 1; }
tail -2 gpurun_out/r6/gpu_tests_ryu4.txt
O=gpurun_out/r6/ryu4.jsonl
: > $O
for c in u2 u3 u1; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --frames 256 --settle-ms 150 --reps 8 --block 8 --arm base: --tag prod >> $O || exit 1
done
for c in u1; do
  LIBIQO_AMD_LIB=$GRAFT_REPO_ROOT/libiqo_amd/variants/ryuexact.so timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --frames 256 --settle-ms 150 --reps 8 --block 8 \
    --arm run: --arm col:ryu_run=0 --tag ryuexact >> $O || exit 1
done
timeout -k 10 200 python scripts/probes/steady_ab.py --config u1 --frames 256 --settle-ms 150 --reps 8 --block 8 --arm base: --tag prod >> $O || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/r6/ryu4.jsonl"):
    d = json.loads(l)
    for k, a in d["arms"].items():
        print(d["tag"], d["config"], d["frames"], k, a["kernel"], a["median_ms"], a["min_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
