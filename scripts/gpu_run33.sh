set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# machine scheduler strategy for kernels.hip: default vs gcn-max-ilp (ilp) vs gcn-max-memory-clause (mcl)
: > $OUT/ab33.txt
for c in c2 g1 g5 c4 c1; do
REPS=2 STEPS=30 BENCH_EXTRA="--config $c --no-probe --alt-frames 0 --no-cpu" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|" "libiqo_amd/variants/ilp.so|" "libiqo_amd/variants/mcl.so|" >> $OUT/ab33.txt 2>&1 || { cat $OUT/ab33.txt; exit 1; }
done
cat $OUT/ab33.txt
