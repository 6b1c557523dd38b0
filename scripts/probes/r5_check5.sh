# Round 5: ryg with 4 columns per thread on wide rows; GPU suite; steady ryg vs walker; host latency.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/r5_pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $OUT/r5_pytest_gpu.log | head; tail -5 $OUT/r5_pytest_gpu.log; exit 1; }
tail -1 $OUT/r5_pytest_gpu.log
SA="timeout -k 10 150 python3 scripts/probes/steady_ab.py --settle-ms 150 --reps 6"
: > $OUT/r5sa_ryg2.jsonl
for c in w1 w3; do
  $SA --config $c --tag $c --arm ryg: --arm walk:ryg=0 >> $OUT/r5sa_ryg2.jsonl 2>> $OUT/r5c5.err || exit 1
done
$SA --config g1 --tag g1 --arm d32: --arm ryg:d32=0 --arm walk:d32=0,ryg=0 >> $OUT/r5sa_ryg2.jsonl 2>> $OUT/r5c5.err || exit 1
bash scripts/gpu_ci.sh hostlat reftool || exit 1
echo done
