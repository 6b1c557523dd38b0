#!/bin/bash
# ryx 2:1: uniform column coefficients + adjacent column pairs (default) vs uniform only (ryx_adj 0)
# vs per-lane tables (ryx_uc 0, ryx_adj 0), steady clock.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; : > $OUT/ab_uc.txt
for c in ${UC_CFGS:-h6 h7 h8 h9}; do
  timeout -k 10 240 python3 scripts/probes/steady_ab.py --config $c --frames 128 --arm adj: --arm uc:ryx_adj=0 --arm lane:ryx_uc=0,ryx_adj=0 >> $OUT/ab_uc.txt 2>&1 || { tail -5 $OUT/ab_uc.txt; exit 1; }
done
python3 scripts/probes/ab_summary.py $OUT/ab_uc.txt
