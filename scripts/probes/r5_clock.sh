# Per-dispatch GPU clock of the C2 kernel: GRBM_GUI_ACTIVE (GPU-busy cycles at the GFX clock)
# over the dispatch's duration, across a bench run's warmup and timed steps (power transient probe).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
timeout -k 10 -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $OUT/r5clk_c2 -o run -- python3 $ROOT/bench.py --config c2 --steps 60 --warmup 5 --no-cpu --no-verify --no-probe --alt-frames 0 > $OUT/r5clk_c2.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/r5tr_c2_drv -o run -- python3 $ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-verify --no-probe > $OUT/r5tr_c2_drv.log 2>&1 &&
tail -1 $OUT/r5tr_c2_drv.log
