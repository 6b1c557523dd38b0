#!/bin/bash
# round 6: C2 XCD chunk size (variant: debug_flags = chunk << 16 on the non-tail path, tail=-1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
O=gpurun_out/r6/c2chunk.jsonl
: > $O
export LIBIQO_AMD_LIB=$GRAFT_REPO_ROOT/libiqo_amd/variants/dbg.so
for f in 256 1024; do
  timeout -k 10 300 python scripts/probes/steady_ab.py --config c2 --frames $f --settle-ms 150 --reps 8 --block 6 \
    --arm default: --arm frame:tail=-1 --arm c45:tail=-1,debug_flags=2949120 --arm c30:tail=-1,debug_flags=1966080 \
    --arm c18:tail=-1,debug_flags=1179648 --arm c9:tail=-1,debug_flags=589824 --arm c180:tail=-1,debug_flags=11796480 >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r6/c2chunk.jsonl"):
    d = json.loads(l)
    for k, a in d["arms"].items():
        print(d["config"], d["frames"], k, a["median_ms"], a["min_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
