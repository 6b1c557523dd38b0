#!/bin/bash
# round 6: C2 frames interleaved over the XCDs (variant debug flag 128) vs contiguous per XCD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
O=gpurun_out/r6/c2inter.jsonl
: > $O
export LIBIQO_AMD_LIB=$GRAFT_REPO_ROOT/libiqo_amd/variants/dbg.so
for f in 256 1024; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --config c2 --frames $f --settle-ms 150 --reps 10 --block 6 \
    --arm contig: --arm inter:debug_flags=128 >> $O || exit 1
done
timeout -k 10 200 python scripts/probes/steady_ab.py --config c3 --frames 64 --settle-ms 150 --reps 8 --block 8 --arm base: >> $O || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/r6/c2inter.jsonl"):
    d = json.loads(l)
    for k, a in d["arms"].items():
        print(d["config"], d["frames"], k, a["kernel"], a["median_ms"], a["min_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
