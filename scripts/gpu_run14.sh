set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# compile-time timing experiments (IQO_SYMB_EXP): e1 no vertical MACs, e2 half the horizontal dots,
# e3 / e4 dot2 / dot4 in place of the MACs; full and compute-only (debug_flags 3)
REPS=2 STEPS=40 BENCH_EXTRA="--no-probe --alt-frames 0 --no-verify" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|" "libiqo_amd/variants/e0.so|" "libiqo_amd/variants/e1.so|" "libiqo_amd/variants/e2.so|" \
  "libiqo_amd/variants/e3.so|" "libiqo_amd/variants/e4.so|" \
  "libiqo_amd/variants/e0.so|--option debug_flags=3" "libiqo_amd/variants/e1.so|--option debug_flags=3" \
  "libiqo_amd/variants/e2.so|--option debug_flags=3" "libiqo_amd/variants/e3.so|--option debug_flags=3" \
  "libiqo_amd/variants/e4.so|--option debug_flags=3" \
  > $OUT/ab14.txt 2>&1 || { cat $OUT/ab14.txt; exit 1; }
cat $OUT/ab14.txt
