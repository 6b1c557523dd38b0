# Round 5: steady-state band count sweep and workgroups per CU (LDS-inflated experiment build) of
# the C2 streamer at 1024 frames per launch.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $ROOT
SA="timeout -k 10 150 python3 scripts/probes/steady_ab.py"
$SA --config c2 --frames 1024 --settle-ms 150 --reps 6 --tag bands --arm base: --arm b24:bands=24 --arm b32:bands=32 --arm b64:bands=64 --arm b96:bands=96 --arm b128:bands=128 --arm b135:bands=135 --arm b270:bands=270 > $OUT/r5sa_bands.json 2> $OUT/r5sa3.err || exit 1
for w in 3 2 1; do
  IQO_EXP_WGCU=$w LIBIQO_AMD_LIB=$ROOT/libiqo_amd/variants/wgcu.so $SA --config c2 --frames 1024 --settle-ms 150 --reps 6 --tag wgcu$w --arm base: --arm b64:bands=64 --arm b128:bands=128 --arm b270:bands=270 >> $OUT/r5sa_wgcu.jsonl 2>> $OUT/r5sa3.err || exit 1
done

# steady-state decomposition of the C2 streamer (variant builds; wrong-output timing arms)
for v in dbgv exp1 exp2; do
  if [ $v = dbgv ]; then ARMS="--arm base: --arm nost:debug_flags=1 --arm noload:debug_flags=2 --arm nomem:debug_flags=3"; else ARMS="--arm base: --arm nomem:debug_flags=3"; fi
  LIBIQO_AMD_LIB=$ROOT/libiqo_amd/variants/$v.so $SA --config c2 --frames 1024 --settle-ms 150 --reps 6 --tag $v $ARMS >> $OUT/r5sa_decomp.jsonl 2>> $OUT/r5sa3.err || exit 1
done
timeout -k 10 200 python3 scripts/probes/pcie_probe.py > $OUT/r5_pcie.json 2>> $OUT/r5sa3.err || exit 1
timeout -k 10 400 python3 scripts/ratio_sweep.py > $OUT/r5_ratio_sweep.txt 2>> $OUT/r5sa3.err || exit 1
echo done2
