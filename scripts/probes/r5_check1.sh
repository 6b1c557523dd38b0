# Round 5: full GPU suite on the current tree, host-pointer latency / reference-tool cycles, default bench line.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/r5_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/r5_pytest_gpu.log; exit 1; }
tail -1 $OUT/r5_pytest_gpu.log
bash scripts/gpu_ci.sh reftool hostlat || exit 1
timeout -k 10 400 python bench.py > $OUT/r5_bench_default.log 2>&1 || { echo "bench failed"; tail -20 $OUT/r5_bench_default.log; exit 1; }
tail -1 $OUT/r5_bench_default.log | cut -c1-400
