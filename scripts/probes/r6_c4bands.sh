#!/bin/bash
# round 6: C4 band / lane sweep at a steady clock; C2 dispatch durations and gaps by batch (rocprof)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
O=gpurun_out/r6/c4bands.jsonl
: > $O
timeout -k 10 200 python scripts/probes/steady_ab.py --config c4 --frames 256 --settle-ms 150 --reps 8 --block 8 \
  --arm b96:bands=96 --arm l48b96:lanes=48,bands=96 --arm l48b144:lanes=48,bands=144 --arm l48b216:lanes=48,bands=216 \
  --arm b144:bands=144 --arm b216:bands=216 --arm l48b288:lanes=48,bands=288 >> $O || exit 1
timeout -k 10 200 python scripts/probes/steady_ab.py --config c4 --frames 64 --settle-ms 150 --reps 8 --block 8 \
  --arm base: --arm b96:bands=96 --arm l48b96:lanes=48,bands=96 --arm l48b144:lanes=48,bands=144 --arm l48b216:lanes=48,bands=216 >> $O || exit 1
cd /tmp && export TMPDIR=/tmp
for f in 64 256 1024; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6/tr_c2_$f -o run -- python3 $GRAFT_REPO_ROOT/scripts/probes/steady_ab.py --config c2 --frames $f --settle-ms 150 --reps 6 --block 8 --arm base: > $GRAFT_REPO_ROOT/gpurun_out/r6/tr_c2_$f.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT
for f in 64 256 1024; do echo "== c2 frames $f"; python scripts/probes/trace_gaps.py $(ls gpurun_out/r6/tr_c2_$f/*kernel_trace.csv | head -1) --skip 40; done
python - <<'PY'
import json
for l in open("gpurun_out/r6/c4bands.jsonl"):
    d = json.loads(l)
    for k, a in d["arms"].items():
        print(d["config"], d["frames"], k, a["median_ms"], a["min_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
