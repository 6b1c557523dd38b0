set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# timing only: the vertical MACs as v_dot2c (512) or v_dot4 (1024) instead of v_pk_mad_u16; full and compute-only (| 3)
REPS=2 STEPS=40 BENCH_EXTRA="--no-probe --alt-frames 0 --no-verify" bash scripts/ab2.sh \
  "libiqo_amd/variants/dbg.so|--option debug_flags=0" "libiqo_amd/variants/dbg.so|--option debug_flags=512" \
  "libiqo_amd/variants/dbg.so|--option debug_flags=1024" "libiqo_amd/variants/dbg.so|--option debug_flags=128" \
  "libiqo_amd/variants/dbg.so|--option debug_flags=3" "libiqo_amd/variants/dbg.so|--option debug_flags=515" \
  "libiqo_amd/variants/dbg.so|--option debug_flags=1027" "libiqo_amd/variants/dbg.so|--option debug_flags=131" \
  > $OUT/ab13.txt 2>&1 || { cat $OUT/ab13.txt; exit 1; }
cat $OUT/ab13.txt
