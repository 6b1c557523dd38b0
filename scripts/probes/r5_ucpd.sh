#!/bin/bash
# Lanczos-8 / -9 2:1 (uniform columns): prefetch depth 2 (shipped) / 4 / 6 (variant builds), steady clock,
# libraries alternated in separate processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; : > $OUT/ab_ucpd.txt
for rep in 1 2; do
  for lib in libiqo_amd/libiqo_hip.so libiqo_amd/variants/ucpd4.so libiqo_amd/variants/ucpd6.so; do
    for c in h8 h9; do
      LIBIQO_AMD_LIB=$PWD/$lib timeout -k 10 240 python3 scripts/probes/steady_ab.py --config $c --frames 128 --tag $(basename $lib .so) --arm base: >> $OUT/ab_ucpd.txt 2>&1 || { tail -5 $OUT/ab_ucpd.txt; exit 1; }
    done
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/ab_ucpd.txt"):
    if l.startswith("{"):
        d = json.loads(l); a = d["arms"]["base"]
        print(d["config"], d["tag"], a["median_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
