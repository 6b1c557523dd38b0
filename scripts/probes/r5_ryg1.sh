#!/bin/bash
# ryg schedule A/Bs at a steady clock: band counts and column parts (W1, W3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT
SA="timeout -k 10 240 python3 scripts/probes/steady_ab.py"
$SA --config w1 --tag w1 --arm base: --arm b3:bands=3 --arm b8:bands=8 --arm b12:bands=12 --arm b24:bands=24 --arm one512:ryx_split=0 > $OUT/ryg1_w1.txt 2>&1 || { tail -5 $OUT/ryg1_w1.txt; exit 1; }
$SA --config w3 --tag w3 --arm base: --arm b3:bands=3 --arm b8:bands=8 --arm b12:bands=12 --arm b24:bands=24 --arm one512:ryx_split=0 > $OUT/ryg1_w3.txt 2>&1 || { tail -5 $OUT/ryg1_w3.txt; exit 1; }
cat $OUT/ryg1_w1.txt $OUT/ryg1_w3.txt
