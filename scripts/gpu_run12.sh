set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# vertical pass instruction order: vo1 = pair sums first, vo2 = v_pk_add_u16 pair sums (bit-exact); full and compute-only (dbg 3)
REPS=2 STEPS=40 BENCH_EXTRA="--no-probe --alt-frames 0" bash scripts/ab2.sh \
  "libiqo_amd/variants/dbg.so|--option debug_flags=0" "libiqo_amd/variants/vo1.so|--option debug_flags=0" \
  "libiqo_amd/variants/vo2.so|--option debug_flags=0" \
  "libiqo_amd/variants/dbg.so|--option debug_flags=3 --no-verify" "libiqo_amd/variants/vo1.so|--option debug_flags=3 --no-verify" \
  "libiqo_amd/variants/vo2.so|--option debug_flags=3 --no-verify" \
  > $OUT/ab12.txt 2>&1 || { cat $OUT/ab12.txt; exit 1; }
cat $OUT/ab12.txt
