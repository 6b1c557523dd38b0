#!/bin/bash
# round 6: two ranks on the one-GPU box (gloo control plane): band mode with per-rank windows, image mode
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
export IQO_BENCH_DIST=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --shard band --frames 64 --steps 10 --warmup 3 --no-cpu > gpurun_out/r6/band2.json 2> gpurun_out/r6/band2.err || { tail -20 gpurun_out/r6/band2.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
  bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu > gpurun_out/r6/image2.json 2> gpurun_out/r6/image2.err || { tail -20 gpurun_out/r6/image2.err; exit 1; }
tail -c 1500 gpurun_out/r6/band2.json; echo; tail -c 600 gpurun_out/r6/image2.json
