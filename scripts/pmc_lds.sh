#!/bin/bash
# LDS / wait counters for one bench config:  CFG=g1 TAG=ld scripts/pmc_lds.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd /tmp || exit 1; export TMPDIR=/tmp
CFG=${CFG:-g1}; TAG=${TAG:-ld}
i=0
for set in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LEVEL_WAVES SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_CYCLES"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/pmc_${TAG}$i" -o run -- python3 "$ROOT/bench.py" --config $CFG --steps 2 --warmup 1 --no-cpu --no-verify ${BENCH_EXTRA} > "$OUT/pmc_${TAG}$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/pmc_${TAG}$i.log"; exit 1; }
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" "$TAG" $i
