#!/bin/bash
# round 6: ryu run mode parity + A/B; C4 new defaults; SQ counters of U2 (ryu run mode)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "ryg or random or golden or linear or padded" > gpurun_out/r6/gpu_tests_ryu2.txt 2>&1 || { tail -40 gpurun_out/r6/gpu_tests_ryu2.txt; exit 1; }
tail -3 gpurun_out/r6/gpu_tests_ryu2.txt
O=gpurun_out/r6/ryu2.jsonl
: > $O
for c in u2 u3; do
  timeout -k 10 200 python scripts/probes/steady_ab.py --config $c --frames 256 --settle-ms 150 --reps 8 --block 8 \
    --arm run: --arm col:ryu_run=0 --arm ryg:ryu=0 >> $O || exit 1
done
timeout -k 10 200 python scripts/probes/steady_ab.py --config c4 --frames 256 --settle-ms 150 --reps 8 --block 8 \
  --arm new: --arm r5:lanes=60,bands=48 >> $O || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/r6/ryu2.jsonl"):
    d = json.loads(l)
    for k, a in d["arms"].items():
        print(d["config"], d["frames"], k, a["kernel"], a["median_ms"], a["min_ms"], a["frac_median"], a["bit_exact_frame0"])
PY
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6/pmc_u2_$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config u2 --steps 2 --warmup 1 --no-cpu --no-verify > $GRAFT_REPO_ROOT/gpurun_out/r6/pmc_u2_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/r6/pmc_u2_$i.log; exit 1; }
done
cd $GRAFT_REPO_ROOT && python3 scripts/pmc_summary.py gpurun_out/r6 pmc_u2_ 2 || true
