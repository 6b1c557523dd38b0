#!/bin/bash
# bench.py --config CFG with --rotate 2 / 3 / 4 alternated on one box (auto warmup).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; : > $OUT/rotate_cfg_ab.txt
for c in ${ROT_CFGS:-c3 c4}; do
  for rep in 1 2; do
    for rot in 2 3 4; do
      timeout -k 10 200 python bench.py --config $c --no-cpu --no-probe --rotate $rot > $OUT/rot.log 2>&1 || { tail -5 $OUT/rot.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('$OUT/rot.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$c rotate $rot', d['ms_per_step'], r['kernel_ms_per_launch'], r['frac'], d['parity'])" >> $OUT/rotate_cfg_ab.txt
    done
  done
done
cat $OUT/rotate_cfg_ab.txt
