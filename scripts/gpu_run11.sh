set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# is C2 VALU-bound?  dbg 128 drops the vertical MACs (-32 VALU / row), 256 half the horizontal
# dots (-24 VALU / row), 3 drops all global memory traffic
REPS=2 STEPS=40 BENCH_EXTRA="--no-probe --alt-frames 0 --no-verify" bash scripts/ab2.sh \
  "libiqo_amd/variants/dbg.so|--option debug_flags=0" "libiqo_amd/variants/dbg.so|--option debug_flags=128" \
  "libiqo_amd/variants/dbg.so|--option debug_flags=256" "libiqo_amd/variants/dbg.so|--option debug_flags=384" \
  "libiqo_amd/variants/dbg.so|--option debug_flags=3" "libiqo_amd/variants/dbg.so|--option debug_flags=131" \
  "libiqo_amd/variants/dbg.so|--option debug_flags=259" "libiqo_amd/variants/dbg.so|--option debug_flags=387" \
  > $OUT/ab11.txt 2>&1 || { cat $OUT/ab11.txt; exit 1; }
cat $OUT/ab11.txt
