set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# ratio-Y kernel with the zero outer row taps trimmed: parity, then old (HEAD) vs new at 9:4
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "ryx or ratio or emul" > $OUT/t34.txt 2>&1 || { tail -30 $OUT/t34.txt; exit 1; }
tail -3 $OUT/t34.txt
: > $OUT/sweep34.txt
for rep in 1 2; do
for v in libiqo_amd/variants/old.so libiqo_amd/libiqo_hip.so libiqo_amd/variants/wpe5.so; do
  echo "== $v rep$rep" >> $OUT/sweep34.txt
  LIBIQO_AMD_LIB=$ROOT/$v timeout -k 10 200 python scripts/ratio_sweep.py --match "x480" >> $OUT/sweep34.txt 2>&1 || { tail -20 $OUT/sweep34.txt; exit 1; }
  LIBIQO_AMD_LIB=$ROOT/$v timeout -k 10 200 python scripts/ratio_sweep.py --match "x320" >> $OUT/sweep34.txt 2>&1 || { tail -20 $OUT/sweep34.txt; exit 1; }
done
done
cat $OUT/sweep34.txt
