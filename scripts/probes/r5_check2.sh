# Round 5: GPU suite on the current tree; host-pointer probes; new streamer band default vs the old one at
# steady clock; Lanczos-8/-9 ryx at 2 waves per SIMD (variant build); the driver's bench command.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/r5_pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $OUT/r5_pytest_gpu.log | head; tail -5 $OUT/r5_pytest_gpu.log; exit 1; }
tail -1 $OUT/r5_pytest_gpu.log
bash scripts/gpu_ci.sh reftool hostlat || exit 1
SA="timeout -k 10 150 python3 scripts/probes/steady_ab.py --settle-ms 150 --reps 6"
$SA --config c2 --frames 1024 --tag c2new --arm base: --arm b50:bands=50 >> $OUT/r5sa_check2.jsonl 2>> $OUT/r5c2.err || exit 1
$SA --config c1 --tag c1new --arm base: --arm b5:bands=5 >> $OUT/r5sa_check2.jsonl 2>> $OUT/r5c2.err || exit 1
for v in default wpe2; do
  if [ $v = default ]; then L=""; else L=$ROOT/libiqo_amd/variants/$v.so; fi
  for c in h8 h9; do
    LIBIQO_AMD_LIB=$L $SA --config $c --tag $v-$c --arm base: >> $OUT/r5sa_check2.jsonl 2>> $OUT/r5c2.err || exit 1
  done
done
for c in w1 w2 w3 u1 g5; do
  $SA --config $c --tag $c --arm base: >> $OUT/r5sa_check2.jsonl 2>> $OUT/r5c2.err || exit 1
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r5_bench_drv.log 2>&1 || { echo "bench failed"; tail -5 $OUT/r5_bench_drv.log; exit 1; }
tail -1 $OUT/r5_bench_drv.log | cut -c1-600
echo done
