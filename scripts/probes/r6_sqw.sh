#!/bin/bash
# round 6: SQ counters of the general-row downscales (W1, W6) and U2 for comparison
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
ROOT=$(pwd); mkdir -p gpurun_out/r6; cd /tmp && export TMPDIR=/tmp
for c in w1 w6; do
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
             "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $ROOT/gpurun_out/r6/pmc_${c}_$i -o run -- python3 $ROOT/bench.py --config $c --steps 2 --warmup 1 --no-cpu --no-verify > $ROOT/gpurun_out/r6/pmc_${c}_$i.log 2>&1 || { echo "pass $c $i failed"; tail -5 $ROOT/gpurun_out/r6/pmc_${c}_$i.log; exit 1; }
  done
done
