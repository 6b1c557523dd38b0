# Round 5: host-pointer latency breakdown (C1 and C2 I420, pageable vs pinned), rocprof kernel stats of the
# driver's bench command (C2, 1024 frames) and its FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $ROOT
bash scripts/gpu_ci.sh hostlat || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2drv -o run -- python3 $ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-probe > $OUT/prof_c2drv.log 2>&1 || { echo "prof failed"; tail -5 $OUT/prof_c2drv.log; exit 1; }
tail -1 $OUT/prof_c2drv.log | cut -c1-300
cd $ROOT
PMC_CFGS=c2 bash scripts/gpu_ci.sh pmc || exit 1
python3 scripts/pmc_to_json.py gpurun_out c2 --round r05
echo done
