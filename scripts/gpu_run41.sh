set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
# ratio-Y kernel: coefficient splats loaded per row (shipped) vs once before the walk (pre)
: > $OUT/sweep41.txt
for rep in 1 2; do
for v in libiqo_amd/libiqo_hip.so libiqo_amd/variants/pre.so; do
  echo "== $v rep$rep" >> $OUT/sweep41.txt
  LIBIQO_AMD_LIB=$ROOT/$v timeout -k 10 200 python scripts/ratio_sweep.py --match "x480" >> $OUT/sweep41.txt 2>&1 || { tail -20 $OUT/sweep41.txt; exit 1; }
done
done
grep -v amdgpu.ids $OUT/sweep41.txt
