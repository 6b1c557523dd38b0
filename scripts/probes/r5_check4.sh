# Round 5: GPU suite with the general-row kernel (ryg) and the direct host path; steady-clock ryg vs the
# walker on the walker shapes; host-pointer latency (direct vs staging pipeline); reference tool cycles.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/r5_pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $OUT/r5_pytest_gpu.log | head; tail -5 $OUT/r5_pytest_gpu.log; exit 1; }
tail -1 $OUT/r5_pytest_gpu.log
SA="timeout -k 10 150 python3 scripts/probes/steady_ab.py --settle-ms 150 --reps 6"
for c in w1 w2 w3; do
  $SA --config $c --tag $c --arm ryg: --arm walk:ryg=0 >> $OUT/r5sa_ryg.jsonl 2>> $OUT/r5c4.err || exit 1
done
bash scripts/gpu_ci.sh hostlat reftool || exit 1
echo done
