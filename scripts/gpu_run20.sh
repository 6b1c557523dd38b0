set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export IQO_REQUIRE_HIP=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pt20.log 2>&1 || { tail -30 $OUT/pt20.log; exit 1; }
tail -1 $OUT/pt20.log
rm -f $OUT/ab19.txt
timeout -k 10 300 bash scripts/gpu_run19.sh > /dev/null 2>&1 || { cat $OUT/ab19.txt; exit 1; }
cat $OUT/ab19.txt
timeout -k 10 400 python bench.py --config c1 --steps 50 --warmup 5 > $OUT/bench_c1.log 2>&1 || { tail -10 $OUT/bench_c1.log; exit 1; }
tail -1 $OUT/bench_c1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["frac"], d["reference_benchmark"])'
