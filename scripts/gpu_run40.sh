set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
# full GPU suite + smoke on the build with the bottom-up 3:2 bands; G1 rocprof stats
bash scripts/gpu_ci.sh tests || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
PROF_CFGS="g1" bash scripts/gpu_ci.sh prof || exit 1
timeout -k 10 300 python bench.py --config g1 --steps 30 --warmup 3 --no-cpu > $OUT/bench_g1.log 2>&1 || { tail -20 $OUT/bench_g1.log; exit 1; }
tail -1 $OUT/bench_g1.log
