#!/bin/bash
# Round-5 end-of-round evidence on one box: GPU suite, steady bench lines of every config, the
# driver's bench command, the same command under rocprofv3 --kernel-trace --stats, the C2 PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
bash scripts/gpu_ci.sh tests || exit 1
BENCH_EXTRA="--warmup 100 --steps 50" bash scripts/gpu_ci.sh benchlines > $OUT/benchlines.txt 2>&1 || { tail -5 $OUT/benchlines.txt; exit 1; }
cp $OUT/bench_lines.jsonl $OUT/bench_lines_steady.jsonl
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 || { tail -5 $OUT/bench_driver.log; exit 1; }
tail -1 $OUT/bench_driver.log > $OUT/bench_driver.json
cd /tmp || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_drv" -o run -- python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu --no-probe > "$OUT/prof_drv.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof_drv.log"; exit 1; }
grep '^{"metric"' "$OUT/prof_drv.log" > "$OUT/bench_line_under_rocprof.json"
cd "$ROOT" || exit 1
PMC_CFGS="c2" bash scripts/gpu_ci.sh pmc || exit 1
python3 scripts/pmc_to_json.py gpurun_out c2 --round r05
cat $OUT/benchlines.txt | tail -30
python3 -c "
import json; d=json.load(open('$OUT/bench_driver.json')); r=d['roofline']
print('driver', d['value'], d['ms_per_step'], r['frac'], r['traffic'], d['cpu_baseline']['value'], d['parity'])"
