set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# frame-stacked streamer on narrow frames: N1 (5 frames per workgroup), N2 (Lanczos-3, 3 per workgroup)
for c in n1 n2; do
REPS=2 STEPS=40 BENCH_EXTRA="--config $c --no-probe --no-cpu" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|" "libiqo_amd/libiqo_hip.so|--option stack=0" \
  >> $OUT/ab19.txt 2>&1 || { cat $OUT/ab19.txt; exit 1; }
done
cat $OUT/ab19.txt
