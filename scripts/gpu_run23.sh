set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export IQO_REQUIRE_HIP=1
timeout -k 10 200 python scripts/probes/host_latency.py > $OUT/host_latency.txt 2>&1 || { tail -5 $OUT/host_latency.txt; exit 1; }
cat $OUT/host_latency.txt
# the reference's own benchmark tool (benchmark/benchmark.cpp, unchanged) linked against the drop-in
B=tests/native/_build/dropin/benchmark
: > $OUT/ref_tool.txt
for args in "-m lanczos2 -iw 640 -ih 480 -ow 320 -oh 240" "-m lanczos3 -iw 3840 -ih 2160 -ow 1920 -oh 1080" \
            "-m area -iw 7680 -ih 4320 -ow 1920 -oh 1080" "-m linear -iw 1920 -ih 1080 -ow 3840 -oh 2160"; do
  echo "== benchmark $args" >> $OUT/ref_tool.txt
  timeout -k 10 120 $B $args >> $OUT/ref_tool.txt 2>&1 || { tail -5 $OUT/ref_tool.txt; exit 1; }
done
cat $OUT/ref_tool.txt
