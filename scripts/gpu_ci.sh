#!/bin/bash
# GPU-box command sequence (run via gpurun from the repo root).  Every GPU step has its own
# time limit and the chain stops at the first failure (no retries on the GPU).
#   scripts/gpu_ci.sh [tests] [bench] [prof] [pmc]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
want() { [[ " $* " == *" all "* ]] || [[ " $ARGS " == *" $1 "* ]]; }
ARGS="$*"
[ -z "$ARGS" ] && ARGS="tests bench"
if want tests; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -20 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
fi
if want bench; then
  for c in c2 c3 c4; do
    timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu ${BENCH_EXTRA} > "$OUT/bench_$c.log" 2>&1 || { echo "bench $c failed"; tail -20 "$OUT/bench_$c.log"; exit 1; }
    tail -1 "$OUT/bench_$c.log"
  done
fi
if want fullbench; then
  timeout -k 10 400 python bench.py > "$OUT/bench_full.log" 2>&1 || { echo "full bench failed"; tail -20 "$OUT/bench_full.log"; exit 1; }
  tail -1 "$OUT/bench_full.log"
fi
if want prof; then
  cd /tmp || exit 1
  for c in ${PROF_CFGS:-c2 c3 c4 g1 g2 g3}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$c" -o run -- python3 "$ROOT/bench.py" --config $c --steps 10 --warmup 2 --no-cpu --no-verify --no-probe --alt-frames 0 > "$OUT/prof_$c.log" 2>&1 || { echo "prof $c failed"; tail -20 "$OUT/prof_$c.log"; exit 1; }
  done
  cd "$ROOT" || exit 1
fi
if want pmc; then
  cd /tmp || exit 1
  for c in ${PMC_CFGS:-c2 c3 c4 g1}; do
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch_$c" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $c --steps 3 --warmup 1 --no-cpu --no-verify --no-probe --alt-frames 0 > "$OUT/pmc_fetch_$c.log" 2>&1 || { echo "pmc fetch $c failed"; tail -20 "$OUT/pmc_fetch_$c.log"; exit 1; }
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write_$c" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $c --steps 3 --warmup 1 --no-cpu --no-verify --no-probe --alt-frames 0 > "$OUT/pmc_write_$c.log" 2>&1 || { echo "pmc write $c failed"; tail -20 "$OUT/pmc_write_$c.log"; exit 1; }
  done
  cd "$ROOT" || exit 1
fi
echo "gpu_ci done"
