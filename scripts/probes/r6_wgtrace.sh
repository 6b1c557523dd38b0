#!/bin/bash
# round 6: workgroup timeline of the C2 streamer (variant build with per-workgroup clock records)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
O=gpurun_out/r6/wgtrace.jsonl
: > $O
export LIBIQO_AMD_LIB=$GRAFT_REPO_ROOT/libiqo_amd/variants/trace.so
for f in 256 1024; do
  timeout -k 10 120 python scripts/probes/wg_trace.py --frames $f --dump gpurun_out/r6/wgtrace_$f.npy >> $O || exit 1
done
timeout -k 10 120 python scripts/probes/wg_trace.py --frames 256 --option tail=-1 --dump gpurun_out/r6/wgtrace_256_notail.npy >> $O || exit 1
timeout -k 10 120 python scripts/probes/wg_trace.py --frames 64 --dump gpurun_out/r6/wgtrace_64.npy >> $O || exit 1
cat $O
