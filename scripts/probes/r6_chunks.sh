#!/bin/bash
# round 6: XCD chunk map (xcd_chunks, production) vs xcd_spread (variant -DIQO_XCD_SPREAD) over the kernel families
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/gpu_tests_chunks.txt 2>&1 || { tail -40 gpurun_out/r6/gpu_tests_chunks.txt; exit 1; }
tail -2 gpurun_out/r6/gpu_tests_chunks.txt
O=gpurun_out/r6/chunks.jsonl
: > $O
for c in g1 g2 g3 g4 g5 h2 w1 w4 w6 u1 u2 u3 c1; do
  for lib in prod spread prod spread; do
    if [ $lib = spread ]; then export LIBIQO_AMD_LIB=$GRAFT_REPO_ROOT/libiqo_amd/variants/spread.so; else unset LIBIQO_AMD_LIB; fi
    timeout -k 10 120 python scripts/probes/steady_ab.py --config $c --settle-ms 100 --reps 4 --block 8 --arm base: --tag $lib >> $O || exit 1
  done
done
unset LIBIQO_AMD_LIB
python - <<'PY'
import json, collections
r = collections.defaultdict(list)
for l in open("gpurun_out/r6/chunks.jsonl"):
    d = json.loads(l); a = d["arms"]["base"]
    r[(d["config"], d["tag"])].append(a["median_ms"])
    assert a["bit_exact_frame0"]
cfgs = sorted({k[0] for k in r})
for c in cfgs:
    p, s = min(r[(c, "prod")]), min(r[(c, "spread")])
    print("%-4s chunks %.4f  spread %.4f  ratio %.3f" % (c, p, s, p / s))
PY
