set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# C1: ring depth (prefetch 3 = 4 slots, 4 = 5 packed, 5 = 8 packed: two window periods) and the
# time split (dbg: 1 stores dropped, 2 loads dropped, 3 both); C2 at ring depth 10
: > $OUT/ab36.txt
REPS=2 STEPS=30 BENCH_EXTRA="--config c1 --no-probe --alt-frames 0 --no-cpu" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|" "libiqo_amd/libiqo_hip.so|--option prefetch=4" "libiqo_amd/libiqo_hip.so|--option prefetch=5" \
  "libiqo_amd/variants/dbg.so|--option debug_flags=1" "libiqo_amd/variants/dbg.so|--option debug_flags=2" "libiqo_amd/variants/dbg.so|--option debug_flags=3" >> $OUT/ab36.txt 2>&1 || { cat $OUT/ab36.txt; exit 1; }
REPS=2 STEPS=20 BENCH_EXTRA="--config c2 --no-probe --alt-frames 0 --no-cpu" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|" "libiqo_amd/libiqo_hip.so|--option prefetch=5" >> $OUT/ab36.txt 2>&1 || { cat $OUT/ab36.txt; exit 1; }
cat $OUT/ab36.txt
