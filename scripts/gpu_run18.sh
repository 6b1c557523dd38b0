set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export IQO_REQUIRE_HIP=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "stack or stream_variants or device_batch or yuv420 or golden" > $OUT/pt18.log 2>&1 || { tail -30 $OUT/pt18.log; exit 1; }
tail -1 $OUT/pt18.log
REPS=2 STEPS=40 BENCH_EXTRA="--config c1 --no-probe --no-cpu" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|" "libiqo_amd/libiqo_hip.so|--option stack=0" \
  "libiqo_amd/libiqo_hip.so|--option rounds=3" "libiqo_amd/libiqo_hip.so|--option rounds=12" \
  > $OUT/ab18.txt 2>&1 || { cat $OUT/ab18.txt; exit 1; }
cat $OUT/ab18.txt
