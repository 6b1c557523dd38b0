set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export IQO_REQUIRE_HIP=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "ryx or golden" > $OUT/pt29.log 2>&1 || { tail -30 $OUT/pt29.log; exit 1; }
tail -1 $OUT/pt29.log
timeout -k 10 300 python scripts/ratio_sweep.py --match "x480" > $OUT/rs29a.txt 2>&1 || { tail -5 $OUT/rs29a.txt; exit 1; }
timeout -k 10 300 python scripts/ratio_sweep.py --match "x480" --opt ryx_split=0 > $OUT/rs29b.txt 2>&1 || { tail -5 $OUT/rs29b.txt; exit 1; }
echo "split:"; grep ryx $OUT/rs29a.txt; echo "one workgroup per row:"; grep ryx $OUT/rs29b.txt
