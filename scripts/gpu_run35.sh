set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# C1 time split (block-shared streamer, stack=0): stores dropped (1), loads dropped (2), both (3)
: > $OUT/ab35.txt
REPS=2 STEPS=30 BENCH_EXTRA="--config c1 --no-probe --alt-frames 0 --no-cpu" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|" "libiqo_amd/variants/dbg.so|--option stack=0" "libiqo_amd/variants/dbg.so|--option stack=0 --option debug_flags=1" \
  "libiqo_amd/variants/dbg.so|--option stack=0 --option debug_flags=2" "libiqo_amd/variants/dbg.so|--option stack=0 --option debug_flags=3" >> $OUT/ab35.txt 2>&1 || { cat $OUT/ab35.txt; exit 1; }
cat $OUT/ab35.txt
