# Round 5: steady-state cache-policy variants of the C2 streamer at 1024 frames per launch, and
# frames per launch (512 / 1024 / 2048) on the default build.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $ROOT
SA="timeout -k 10 150 python3 scripts/probes/steady_ab.py"
for f in 512 2048; do
  $SA --config c2 --frames $f --settle-ms 150 --tag frames$f --arm base: >> $OUT/r5sa_frames.jsonl 2>> $OUT/r5sa2.err || exit 1
done
for rep in 1 2; do
  for v in default st18 st16 st3 ld1 ld2; do
    if [ $v = default ]; then L=""; else L=$ROOT/libiqo_amd/variants/$v.so; fi
    LIBIQO_AMD_LIB=$L $SA --config c2 --frames 1024 --settle-ms 150 --reps 6 --tag $v --arm base: >> $OUT/r5sa_pol.jsonl 2>> $OUT/r5sa2.err || exit 1
  done
done
echo done
