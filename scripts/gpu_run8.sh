set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export IQO_REQUIRE_HIP=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "1024_frame or 256_frame" > $OUT/pt8.log 2>&1 || { tail -30 $OUT/pt8.log; exit 1; }
tail -1 $OUT/pt8.log
# C2 time decomposition on fresh batches: debug_flags 1 = no stores, 2 = no source loads, 3 = neither
REPS=2 STEPS=40 BENCH_EXTRA="--no-probe --alt-frames 0 --no-verify" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|" "libiqo_amd/variants/dbg.so|--option debug_flags=1" \
  "libiqo_amd/variants/dbg.so|--option debug_flags=2" "libiqo_amd/variants/dbg.so|--option debug_flags=3" \
  "libiqo_amd/variants/dbg.so|--option debug_flags=0" > $OUT/ab8.txt 2>&1 || { cat $OUT/ab8.txt; exit 1; }
cat $OUT/ab8.txt
CFG=c2 TAG=sqc2 bash scripts/pmc_sq.sh > $OUT/sq_c2.txt 2>&1 || { tail -5 $OUT/sq_c2.txt; exit 1; }
cat $OUT/sq_c2.txt
cd /tmp
for n in 128 256 1024; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2_f$n -o run -- python3 $ROOT/bench.py --frames $n --steps 20 --warmup 3 --no-cpu --no-verify --no-probe --alt-frames 0 > $OUT/prof_c2_f$n.log 2>&1 || { tail -5 $OUT/prof_c2_f$n.log; exit 1; }
  tail -1 $OUT/prof_c2_f$n.log | cut -c1-400
done
cd $ROOT
timeout -k 10 400 python bench.py --config c1 --steps 50 --warmup 5 > $OUT/bench_c1.log 2>&1 || { tail -10 $OUT/bench_c1.log; exit 1; }
tail -1 $OUT/bench_c1.log
