set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# round-end rehearsal on the final build: full GPU suite, smoke, default bench line; G5 / G2 rocprof + PMC
bash scripts/gpu_ci.sh tests fullbench || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
PROF_CFGS="g5" PMC_CFGS="g5" bash scripts/gpu_ci.sh prof pmc || exit 1
timeout -k 10 300 python bench.py --config g5 --steps 20 --warmup 3 --no-cpu > $OUT/bench_g5.log 2>&1 || { tail -20 $OUT/bench_g5.log; exit 1; }
tail -1 $OUT/bench_g5.log
