set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# C1 time split, one frame per workgroup (stack=0) vs three (stack=2): 1 no stores, 2 no loads, 3 neither
: > $OUT/ab38.txt
REPS=2 STEPS=30 BENCH_EXTRA="--config c1 --no-probe --alt-frames 0 --no-cpu" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|--option stack=2" \
  "libiqo_amd/variants/dbg.so|--option stack=2 --option debug_flags=1" "libiqo_amd/variants/dbg.so|--option stack=2 --option debug_flags=2" \
  "libiqo_amd/variants/dbg.so|--option stack=2 --option debug_flags=3" "libiqo_amd/libiqo_hip.so|--option stack=2 --option rounds=2" \
  "libiqo_amd/libiqo_hip.so|--option stack=2 --option rounds=12" "libiqo_amd/libiqo_hip.so|" >> $OUT/ab38.txt 2>&1 || { cat $OUT/ab38.txt; exit 1; }
cat $OUT/ab38.txt
