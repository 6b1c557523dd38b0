set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
# 3:2 kernel with odd bands walking bottom-up: parity, G1 A/B (ratio_alt 1 = default vs 0), G1 PMC
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "d32 or golden or ratio" > $OUT/t39.txt 2>&1 || { tail -30 $OUT/t39.txt; exit 1; }
tail -2 $OUT/t39.txt
: > $OUT/ab39.txt
REPS=3 STEPS=30 BENCH_EXTRA="--config g1 --no-probe --alt-frames 0 --no-cpu" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|" "libiqo_amd/libiqo_hip.so|--option ratio_alt=0" >> $OUT/ab39.txt 2>&1 || { cat $OUT/ab39.txt; exit 1; }
cat $OUT/ab39.txt
PMC_CFGS="g1" bash scripts/gpu_ci.sh pmc || exit 1
