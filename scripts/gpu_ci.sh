#!/bin/bash
# GPU-box command sequence (run via gpurun from the repo root).  Every GPU step has its own
# time limit and the chain stops at the first failure (no retries on the GPU).
#   scripts/gpu_ci.sh TARGET...        (default: tests bench)
# Targets (environment knobs in brackets):
#   tests       pytest -m gpu, one process                      [PYTEST_K: -k expression]
#   smoke       __graft_entry__.smoke()
#   bench       short bench lines per config                    [CFGS, default "c2 c3 c4"; BENCH_EXTRA]
#   fullbench   the driver's default `python bench.py`
#   benchlines  one 30-step bench line per config into gpurun_out/bench_lines.jsonl [CFGS, default all]
#   prof        rocprofv3 --kernel-trace --stats per config     [PROF_CFGS]
#   pmc         FETCH_SIZE / WRITE_SIZE passes per config        [PMC_CFGS]
#   sq          SQ / GRBM counter passes (scripts/pmc_sq.sh)     [SQ_CFGS, BENCH_EXTRA]
#   ab          interleaved A/B of library variants / options   [AB: arms separated by ";;", each
#               "lib.so|bench args" (scripts/ab2.sh); REPS, STEPS, BENCH_EXTRA; AB_OUT file name]
#   sweep       scripts/ratio_sweep.py                           [SWEEP_ARGS]
#   reftool     the reference's own benchmark (compiled unchanged against this library) on the
#               four BASELINE shapes, I420, resizers constructed in the timed loop
#   hostlat     scripts/probes/host_latency.py
# Results go to gpurun_out/ (copied into profiles/rNN/ by hand when they are committed).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="$*"
[ -z "$ARGS" ] && ARGS="tests bench"
ALLCFGS="c1 c2 c3 c4 g1 g2 g3 g4 g5 g6 n1 n2 h1 h2 h3 h4 h5 h6 h7 h8 h9 w1 w2 w3 w4 w5 w6 w7 u1 u2 u3"
for target in $ARGS; do
case $target in
tests)
  K=()
  [ -n "$PYTEST_K" ] && K=(-k "$PYTEST_K")
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${K[@]}" > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
  ;;
smoke)
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
  ;;
bench)
  for c in ${CFGS:-c2 c3 c4}; do
    timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu ${BENCH_EXTRA} > "$OUT/bench_$c.log" 2>&1 || { echo "bench $c failed"; tail -20 "$OUT/bench_$c.log"; exit 1; }
    tail -1 "$OUT/bench_$c.log"
  done
  ;;
fullbench)
  timeout -k 10 400 python bench.py > "$OUT/bench_full.log" 2>&1 || { echo "full bench failed"; tail -20 "$OUT/bench_full.log"; exit 1; }
  tail -1 "$OUT/bench_full.log"
  ;;
benchlines)
  : > "$OUT/bench_lines.jsonl"
  for c in ${CFGS:-$ALLCFGS}; do
    timeout -k 10 300 python bench.py --config $c --steps 30 --warmup 3 --no-cpu --no-probe ${BENCH_EXTRA} > "$OUT/bl_$c.log" 2>&1 || { echo "bench $c failed"; tail -5 "$OUT/bl_$c.log"; exit 1; }
    tail -1 "$OUT/bl_$c.log" >> "$OUT/bench_lines.jsonl"
  done
  python3 -c "
import json
for l in open('$OUT/bench_lines.jsonl'):
    d = json.loads(l); r = d['roofline']
    print('%-44s %-40s %8.4f ms  frac %.3f' % (d['config']['workload'][:44], r.get('kernel', '')[:40], r['kernel_ms_per_launch'], r['frac']))"
  ;;
prof)
  cd /tmp || exit 1
  for c in ${PROF_CFGS:-c2 c3 c4 g1 g2 g3}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$c" -o run -- python3 "$ROOT/bench.py" --config $c --steps 40 --warmup 5 --no-cpu --no-verify --no-probe --alt-frames 0 > "$OUT/prof_$c.log" 2>&1 || { echo "prof $c failed"; tail -20 "$OUT/prof_$c.log"; exit 1; }
  done
  cd "$ROOT" || exit 1
  ;;
pmc)
  cd /tmp || exit 1
  for c in ${PMC_CFGS:-c2 c3 c4 g1}; do
    timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch_$c" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $c --steps 3 --warmup 1 --no-cpu --no-verify --no-probe --alt-frames 0 > "$OUT/pmc_fetch_$c.log" 2>&1 || { echo "pmc fetch $c failed"; tail -20 "$OUT/pmc_fetch_$c.log"; exit 1; }
    timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write_$c" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $c --steps 3 --warmup 1 --no-cpu --no-verify --no-probe --alt-frames 0 > "$OUT/pmc_write_$c.log" 2>&1 || { echo "pmc write $c failed"; tail -20 "$OUT/pmc_write_$c.log"; exit 1; }
  done
  cd "$ROOT" || exit 1
  ;;
sq)
  for c in ${SQ_CFGS:-c2}; do
    CFG=$c TAG=sq_$c bash scripts/pmc_sq.sh > "$OUT/sq_$c.txt" 2>&1 || { echo "sq $c failed"; tail -20 "$OUT/sq_$c.txt"; exit 1; }
    cat "$OUT/sq_$c.txt"
  done
  ;;
ab)
  IFS=$'\n' read -r -d '' -a ARMS < <(printf '%s' "$AB" | sed 's/;;/\n/g'; printf '\0')
  bash scripts/ab2.sh "${ARMS[@]}" > "$OUT/${AB_OUT:-ab.txt}" 2>&1 || { echo "ab failed"; cat "$OUT/${AB_OUT:-ab.txt}"; exit 1; }
  cat "$OUT/${AB_OUT:-ab.txt}"
  ;;
sweep)
  timeout -k 10 400 python scripts/ratio_sweep.py ${SWEEP_ARGS} > "$OUT/ratio_sweep.txt" 2>&1 || { echo "sweep failed"; tail -5 "$OUT/ratio_sweep.txt"; exit 1; }
  cat "$OUT/ratio_sweep.txt"
  ;;
reftool)
  B=tests/native/_build/dropin/benchmark
  : > "$OUT/ref_tool.txt"
  for a in "-m lanczos2 -iw 640 -ih 480 -ow 320 -oh 240" "-m lanczos3 -iw 3840 -ih 2160 -ow 1920 -oh 1080" \
           "-m area -iw 7680 -ih 4320 -ow 1920 -oh 1080" "-m linear -iw 1920 -ih 1080 -ow 3840 -oh 2160"; do
    echo "== benchmark $a" >> "$OUT/ref_tool.txt"
    IQO_REQUIRE_HIP=1 timeout -k 10 120 $B $a >> "$OUT/ref_tool.txt" 2>&1 || { echo "reftool failed"; tail -5 "$OUT/ref_tool.txt"; exit 1; }
  done
  grep -E "^==|elapsed" "$OUT/ref_tool.txt"
  ;;
hostlat)
  timeout -k 10 200 python scripts/probes/host_latency.py > "$OUT/host_latency.txt" 2>&1 || { echo "hostlat failed"; tail -5 "$OUT/host_latency.txt"; exit 1; }
  cat "$OUT/host_latency.txt"
  ;;
*)
  echo "unknown target $target"; exit 2
  ;;
esac
done
echo "gpu_ci done"
