set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# ratio-Y kernel column split: two 4-wave workgroups per row (ryx_split 1, default) vs four 2-wave (2)
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "ryx" > $OUT/t43.txt 2>&1 || { tail -30 $OUT/t43.txt; exit 1; }
tail -2 $OUT/t43.txt
: > $OUT/sweep43.txt
for rep in 1 2; do
for sp in 1 2; do
  echo "== ryx_split=$sp rep$rep" >> $OUT/sweep43.txt
  timeout -k 10 200 python scripts/ratio_sweep.py --match "x480" --opt ryx_split=$sp >> $OUT/sweep43.txt 2>&1 || { tail -20 $OUT/sweep43.txt; exit 1; }
done
done
grep -v amdgpu.ids $OUT/sweep43.txt
