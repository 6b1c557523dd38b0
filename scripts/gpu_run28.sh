set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export IQO_REQUIRE_HIP=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pt28.log 2>&1 || { tail -30 $OUT/pt28.log; exit 1; }
tail -1 $OUT/pt28.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
# C2: where the next DMA is issued within an iteration (0 after the barrier, 1 after the vertical pass, 2 after the horizontal pass)
REPS=3 STEPS=40 BENCH_EXTRA="--no-probe --alt-frames 0 --no-cpu" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|" "libiqo_amd/variants/da1.so|" "libiqo_amd/variants/da2.so|" \
  > $OUT/ab28.txt 2>&1 || { cat $OUT/ab28.txt; exit 1; }
cat $OUT/ab28.txt
