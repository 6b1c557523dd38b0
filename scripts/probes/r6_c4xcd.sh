#!/bin/bash
# round 6: C4 XCD-aware block order (A/B in the variant build), W6 band counts, C4 traffic on the new order
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
O=gpurun_out/r6/c4xcd.jsonl
: > $O
LIBIQO_AMD_LIB=$GRAFT_REPO_ROOT/libiqo_amd/variants/dbg.so timeout -k 10 200 python scripts/probes/steady_ab.py --config c4 --frames 256 --settle-ms 150 --reps 8 --block 8 \
  --arm xcd: --arm plain:debug_flags=64 --tag variant >> $O || exit 1
timeout -k 10 200 python scripts/probes/steady_ab.py --config c4 --frames 256 --settle-ms 150 --reps 8 --block 8 \
  --arm xcd: --arm b144:bands=144 --arm b270:bands=270 --tag prod >> $O || exit 1
timeout -k 10 200 python scripts/probes/steady_ab.py --config w6 --frames 128 --settle-ms 150 --reps 8 --block 8 \
  --arm base: --arm b4:bands=4 --arm b6:bands=6 --arm b9:bands=9 --arm b12:bands=12 --arm b18:bands=18 --tag prod >> $O || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/r6/c4xcd.jsonl"):
    d = json.loads(l)
    for k, a in d["arms"].items():
        print(d["tag"], d["config"], d["frames"], k, a["kernel"], a["median_ms"], a["min_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
PMC_CFGS="c4" bash scripts/gpu_ci.sh pmc || exit 1
python3 scripts/pmc_to_json.py gpurun_out c4 --round r06 && cp profiles/pmc_c4.json gpurun_out/r6/pmc_c4_xcd.json
