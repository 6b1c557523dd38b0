#!/bin/bash
# The driver's bench command with 2 and 3 rotated C2 batches, alternated (one box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
OUT=gpurun_out; mkdir -p $OUT; : > $OUT/rotate_ab.txt
for rep in 1 2 3; do
  for rot in 2 3; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-probe --rotate $rot > $OUT/rot.log 2>&1 || { tail -5 $OUT/rot.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/rot.log').read().strip().splitlines()[-1]); r=d['roofline']
print('rotate $rot', d['ms_per_step'], r['kernel_ms_per_launch'], r['frac'], d['parity'])" >> $OUT/rotate_ab.txt
  done
done
cat $OUT/rotate_ab.txt
