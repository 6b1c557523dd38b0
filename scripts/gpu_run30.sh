set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export IQO_REQUIRE_HIP=1
: > $OUT/bench_lines30.jsonl
for c in c1 c2 c3 c4 g1 g2 g3 g4 g5 g6 n1 n2; do
  timeout -k 10 300 python bench.py --config $c --steps 30 --warmup 3 --no-cpu --no-probe > $OUT/b30_$c.log 2>&1 || { tail -5 $OUT/b30_$c.log; exit 1; }
  tail -1 $OUT/b30_$c.log >> $OUT/bench_lines30.jsonl
done
python3 -c "
import json
for l in open('$OUT/bench_lines30.jsonl'):
    d=json.loads(l); r=d['roofline']
    print('%-45s %-16s %8.4f ms  frac %.4f  %s' % (d['config']['workload'][:45], d['config']['kernel'], r['kernel_ms_per_launch'], r['frac'], d['parity'][:9]))
"
PROF_CFGS="c1 c3 c4 g1 g2 g3 g5" PMC_CFGS="c1 c3 c4 g1 g2 g3" bash scripts/gpu_ci.sh prof pmc > $OUT/ci30.log 2>&1 || { tail -5 $OUT/ci30.log; exit 1; }
tail -1 $OUT/ci30.log
