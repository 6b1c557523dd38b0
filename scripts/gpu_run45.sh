set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
# 3:1 kernel with odd bands walking bottom-up: full GPU suite, smoke, G4 A/B (ratio_alt 1 vs 0), G4 PMC
bash scripts/gpu_ci.sh tests || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
: > $OUT/ab45.txt
REPS=2 STEPS=30 BENCH_EXTRA="--config g4 --no-probe --alt-frames 0 --no-cpu" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|" "libiqo_amd/libiqo_hip.so|--option ratio_alt=0" >> $OUT/ab45.txt 2>&1 || { cat $OUT/ab45.txt; exit 1; }
cat $OUT/ab45.txt
PMC_CFGS="g4" bash scripts/gpu_ci.sh pmc || exit 1
