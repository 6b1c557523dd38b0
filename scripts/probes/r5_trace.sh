set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/r5tr_c2_rot2 -o run -- python3 $ROOT/bench.py --config c2 --steps 60 --warmup 5 --no-cpu --no-verify --no-probe --alt-frames 0 > $OUT/r5tr_c2_rot2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/r5tr_c2_rot5 -o run -- python3 $ROOT/bench.py --config c2 --steps 60 --warmup 5 --no-cpu --no-verify --no-probe --alt-frames 0 --rotate 5 > $OUT/r5tr_c2_rot5.log 2>&1 &&
tail -1 $OUT/r5tr_c2_rot2.log && tail -1 $OUT/r5tr_c2_rot5.log
