#!/bin/bash
# round 6 evidence: GPU suite, smoke, the driver's bench command, its rocprof kernel trace + stats,
# C2 HBM traffic passes, the default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r6f; mkdir -p $OUT
bash scripts/gpu_ci.sh tests smoke > $OUT/ci.txt 2>&1 || { tail -30 $OUT/ci.txt; exit 1; }
cp gpurun_out/pytest_gpu.log $OUT/gpu_tests.txt; cp gpurun_out/smoke.log $OUT/smoke.txt
tail -3 $OUT/ci.txt
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver_cmd.err || { tail -20 $OUT/bench_driver_cmd.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_driver_cmd -o run -- python3 $ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-probe > $OUT/trace_driver_cmd.json 2> $OUT/trace_driver_cmd.err || { tail -20 $OUT/trace_driver_cmd.err; exit 1; }
cd $ROOT
python3 scripts/trace_summary.py $(ls $OUT/trace_driver_cmd/*kernel_trace.csv | head -1) $OUT/trace_driver_cmd.json --steps 20 --warmup 5 --kernel lanczos_symb > $OUT/trace_summary.txt 2>&1 || true
PMC_CFGS="c2 w6" bash scripts/gpu_ci.sh pmc > $OUT/pmc.txt 2>&1 || { tail -20 $OUT/pmc.txt; exit 1; }
python3 scripts/pmc_to_json.py gpurun_out c2 --round r06 > $OUT/pmc_c2_line.txt && cp profiles/pmc_c2.json $OUT/pmc_c2.json && python3 scripts/pmc_to_json.py gpurun_out w6 --round r06 >> $OUT/pmc_c2_line.txt && cp profiles/pmc_w6.json $OUT/pmc_w6.json
timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python3 - <<'PY'
import json
for f in ("bench_driver_cmd.json", "trace_driver_cmd.json", "bench_default.json"):
    d = json.loads(open("gpurun_out/r6f/" + f).read().strip().splitlines()[-1])
    r = d["roofline"]; b = d.get("batch_alt", {}); s = d.get("secondary", {})
    print(f, "frac %.4f ms %.4f alt %s c3 %s c4 %s" % (r["frac"], r["kernel_ms_per_launch"], b.get("frac"),
          s.get("c3", {}).get("frac"), s.get("c4", {}).get("frac")))
PY
cat $OUT/trace_summary.txt | head -12; cat $OUT/pmc_c2_line.txt
