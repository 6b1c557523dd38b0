set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# G5 (ryx, Lanczos-3 1080p -> 854x480): source loads dropped (rx1), stores dropped (rx2)
REPS=2 STEPS=40 BENCH_EXTRA="--config g5 --no-probe --no-verify --no-cpu" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|" "libiqo_amd/variants/rx1.so|" "libiqo_amd/variants/rx2.so|" "libiqo_amd/variants/rx3.so|" \
  > $OUT/ab17.txt 2>&1 || { cat $OUT/ab17.txt; exit 1; }
cat $OUT/ab17.txt
