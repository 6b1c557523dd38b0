set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export IQO_REQUIRE_HIP=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "ryx or golden or native_library or stream_variants" > $OUT/pt16.log 2>&1 || { tail -30 $OUT/pt16.log; exit 1; }
tail -1 $OUT/pt16.log
timeout -k 10 300 python scripts/ratio_sweep.py --match "x480" > $OUT/rs16.txt 2>&1 || { tail -5 $OUT/rs16.txt; exit 1; }
cat $OUT/rs16.txt
