set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export IQO_REQUIRE_HIP=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "host_pointer or yuv420 or concurrent or cpp_dropin or sample or reference_" > $OUT/pt25.log 2>&1 || { tail -30 $OUT/pt25.log; exit 1; }
tail -1 $OUT/pt25.log
B=tests/native/_build/dropin/benchmark
: > $OUT/ref_tool25.txt
for args in "-m lanczos2 -iw 640 -ih 480 -ow 320 -oh 240" "-m lanczos3 -iw 3840 -ih 2160 -ow 1920 -oh 1080" \
            "-m area -iw 7680 -ih 4320 -ow 1920 -oh 1080" "-m linear -iw 1920 -ih 1080 -ow 3840 -oh 2160"; do
  echo "== benchmark $args: $(timeout -k 10 120 $B $args 2>&1 | grep elapsed)" >> $OUT/ref_tool25.txt || { cat $OUT/ref_tool25.txt; exit 1; }
done
cat $OUT/ref_tool25.txt
