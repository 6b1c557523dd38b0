#!/bin/bash
# Steady-clock A/B of two library builds, alternated in separate processes: LIB_A (default: the
# in-tree library) vs LIB_B, for the configs in AB_CFGS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; : > $OUT/lib_ab.txt
A=${LIB_A:-libiqo_amd/libiqo_hip.so}; B=${LIB_B:-libiqo_amd/variants/r5start.so}
for rep in 1 2; do
  for lib in $A $B; do
    for c in ${AB_CFGS:-g2 h4}; do
      LIBIQO_AMD_LIB=$PWD/$lib timeout -k 10 240 python3 scripts/probes/steady_ab.py --config $c --tag $(basename $lib .so) --arm base: >> $OUT/lib_ab.txt 2>&1 || { tail -5 $OUT/lib_ab.txt; exit 1; }
    done
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/lib_ab.txt"):
    if l.startswith("{"):
        d = json.loads(l); a = d["arms"]["base"]
        print(d["config"], d["tag"], a["kernel"], a["median_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
