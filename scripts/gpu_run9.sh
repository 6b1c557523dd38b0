set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export IQO_REQUIRE_HIP=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pt9.log 2>&1 || { tail -30 $OUT/pt9.log; exit 1; }
tail -1 $OUT/pt9.log
# C2 ring depth 5 (= the window period: compile-time ring slots) vs 4; band counts at 128 and 256 frames
REPS=2 STEPS=40 BENCH_EXTRA="--no-probe --alt-frames 0 --no-verify" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|" "libiqo_amd/libiqo_hip.so|--option prefetch=4 --option ring_pack=1" \
  "libiqo_amd/libiqo_hip.so|--option ring_pack=1" \
  "libiqo_amd/libiqo_hip.so|--option prefetch=4 --option ring_pack=1 --bands 24" \
  "libiqo_amd/libiqo_hip.so|--option prefetch=4 --option ring_pack=1 --bands 32" \
  "libiqo_amd/libiqo_hip.so|--option prefetch=4 --option ring_pack=1 --option rounds=4" \
  "libiqo_amd/libiqo_hip.so|--option prefetch=4 --option ring_pack=1 --option rounds=8" \
  "libiqo_amd/libiqo_hip.so|--frames 256" "libiqo_amd/libiqo_hip.so|--frames 256 --option prefetch=4 --option ring_pack=1" \
  "libiqo_amd/libiqo_hip.so|--frames 256 --option prefetch=4 --option ring_pack=1 --option rounds=8" \
  "libiqo_amd/libiqo_hip.so|--frames 256 --option prefetch=4 --option ring_pack=1 --option rounds=12" \
  > $OUT/ab9.txt 2>&1 || { cat $OUT/ab9.txt; exit 1; }
cat $OUT/ab9.txt
