# Round 5: steady-state A/B (settle phase, interleaved blocks) of the C2 streamer's band count,
# tail split, XCD order and cache policies; driver-like trace at 1024 frames per launch.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $ROOT
SA="timeout -k 10 120 python3 scripts/probes/steady_ab.py"
$SA --config c2 --settle-ms 120 --trace --tag opts256 --arm base: --arm r4:rounds=4 --arm r8:rounds=8 --arm r12:rounds=12 --arm tailoff:tail=-1 --arm xcd0:xcd_order=0 > $OUT/r5sa_opts256.json 2> $OUT/r5sa.err &&
$SA --config c2 --frames 1024 --settle-ms 120 --trace --tag opts1024 --arm base: --arm r4:rounds=4 --arm r8:rounds=8 --arm tailoff:tail=-1 > $OUT/r5sa_opts1024.json 2>> $OUT/r5sa.err &&
for rep in 1 2; do
  for v in default nt3 nt0; do
    if [ $v = default ]; then L=""; else L=$ROOT/libiqo_amd/variants/$v.so; fi
    LIBIQO_AMD_LIB=$L $SA --config c2 --settle-ms 120 --tag $v --arm base: --arm r8:rounds=8 >> $OUT/r5sa_nt.jsonl 2>> $OUT/r5sa.err || exit 1
  done
done &&
cd /tmp &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/r5tr_c2_f1024 -o run -- python3 $ROOT/bench.py --frames 1024 --steps 20 --warmup 5 --no-cpu --no-verify --no-probe --alt-frames 0 > $OUT/r5tr_c2_f1024.log 2>&1 &&
tail -1 $OUT/r5tr_c2_f1024.log | cut -c1-300
