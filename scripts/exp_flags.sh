#!/bin/bash
# timing experiments for the Lanczos streamer: debug flags and band counts
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for f in 0 1 2 3 4 7; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu --no-verify --debug-flags $f > gpurun_out/exp_f$f.log 2>&1 || exit 1
  echo "flags=$f $(tail -1 gpurun_out/exp_f$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["roofline"]["kernel_ms_per_launch"])')"
done
for b in 4 8 32 64; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu --no-verify --bands $b > gpurun_out/exp_b$b.log 2>&1 || exit 1
  echo "bands=$b $(tail -1 gpurun_out/exp_b$b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["roofline"]["kernel_ms_per_launch"])')"
done
