#!/bin/bash
# SQ counters for the C2 kernel (separate passes; kernel-trace only beside --pmc)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd /tmp || exit 1; export TMPDIR=/tmp
CFG=${CFG:-c2}
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/pmc_sq$i" -o run -- python3 "$ROOT/bench.py" --config $CFG --steps 2 --warmup 1 --no-cpu --no-verify ${BENCH_EXTRA} > "$OUT/pmc_sq$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/pmc_sq$i.log"; exit 1; }
done
echo done
