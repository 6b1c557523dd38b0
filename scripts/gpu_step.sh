set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gputests.log 2>&1; rc=$?; tail -3 gpurun_out/gputests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for pd in 1 2 3; do timeout -k 10 120 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu --no-verify --prefetch $pd 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('pd', $pd, d['value'], d['roofline']['kernel_ms_per_launch'], d['roofline']['frac'])" || exit 1; done
