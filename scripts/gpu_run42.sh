set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# 3:2 kernel register budget: 4 waves/SIMD (shipped) vs 5 / 6 (variant builds, spilling)
: > $OUT/ab42.txt
REPS=2 STEPS=30 BENCH_EXTRA="--config g1 --no-probe --alt-frames 0 --no-cpu" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|" "libiqo_amd/variants/w5.so|" "libiqo_amd/variants/w6.so|" >> $OUT/ab42.txt 2>&1 || { cat $OUT/ab42.txt; exit 1; }
cat $OUT/ab42.txt
