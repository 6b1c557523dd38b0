#!/bin/bash
# SQ counters for one bench config (separate passes; kernel-trace only beside --pmc).
#   CFG=c2 BENCH_EXTRA="--prefetch 2" TAG=x scripts/pmc_sq.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd /tmp || exit 1; export TMPDIR=/tmp
CFG=${CFG:-c2}; TAG=${TAG:-sq}
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_INST_CYCLES_SALU SQ_CYCLES SQ_BUSY_CU_CYCLES" \
           "SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_IFETCH_LEVEL SQ_LEVEL_WAVES SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/pmc_${TAG}$i" -o run -- python3 "$ROOT/bench.py" --config $CFG --steps 2 --warmup 1 --no-cpu --no-verify ${BENCH_EXTRA} > "$OUT/pmc_${TAG}$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/pmc_${TAG}$i.log"; exit 1; }
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" "$TAG" $i
