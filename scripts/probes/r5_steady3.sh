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
echo done
