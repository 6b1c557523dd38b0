# Round 5: C2 streamer option check at steady clock (90-band default); rocprof stats and HBM counters of the
# driver's bench command; one steady-state bench line per config (100 warmup launches).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $ROOT
SA="timeout -k 10 150 python3 scripts/probes/steady_ab.py --settle-ms 150 --reps 6"
$SA --config c2 --frames 1024 --tag c2opts90 --arm base: --arm pf2:prefetch=2 --arm tailoff:tail=-1 --arm xcd0:xcd_order=0 --arm b80:bands=80 --arm b99:bands=99 > $OUT/r5sa_c2opts90.json 2>> $OUT/r5f1.err || exit 1
$SA --config w1 --tag w1split --arm base: --arm one512:ryx_split=0 > $OUT/r5sa_w1split.json 2>> $OUT/r5f1.err || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2drv -o run -- python3 $ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-probe > $OUT/prof_c2drv.log 2>&1 || { echo "prof failed"; tail -5 $OUT/prof_c2drv.log; exit 1; }
tail -1 $OUT/prof_c2drv.log | cut -c1-300
cd $ROOT
rm -rf $OUT/pmc_fetch_c2 $OUT/pmc_write_c2
PMC_CFGS=c2 bash scripts/gpu_ci.sh pmc || exit 1
BENCH_EXTRA="--steps 50 --warmup 100" bash scripts/gpu_ci.sh benchlines || exit 1
echo done
