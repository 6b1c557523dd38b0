#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
for f in 128 256 512 1024; do
for opt in "" "--option chunk_frames=128" "--option xcd_order=0" "--option chunk_frames=64"; do
  timeout -k 10 120 python bench.py --config c2 --frames $f --steps 20 --warmup 3 --no-cpu --no-probe --no-verify $opt > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "frames $f [$opt] $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel_ms_per_launch"], round(r["kernel_ms_per_launch"]/d["config"]["frames_per_gpu"],6), r["frac"])')"
done
done
