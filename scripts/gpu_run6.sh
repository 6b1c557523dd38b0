set -o pipefail
cd $GRAFT_REPO_ROOT
export IQO_REQUIRE_HIP=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "d31 or area_int or ryx or stream_variants or native_library" > gpurun_out/pt6.log 2>&1 || { tail -30 gpurun_out/pt6.log; exit 1; }
tail -2 gpurun_out/pt6.log
REPS=2 STEPS=30 BENCH_EXTRA="--no-probe --alt-frames 0 --no-verify" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|--option sweep=0" "libiqo_amd/libiqo_hip.so|--option sweep=1" \
  "libiqo_amd/variants/nts0.so|--option sweep=1" "libiqo_amd/variants/ntl0.so|--option sweep=1" \
  "libiqo_amd/variants/nt00.so|--option sweep=1" "libiqo_amd/variants/dbg.so|--option sweep=1 --option debug_flags=4" \
  "libiqo_amd/variants/dbg.so|--option sweep=0 --option debug_flags=4" \
  "libiqo_amd/variants/m1.so|--option sweep=1" "libiqo_amd/variants/m1.so|--option sweep=0 --option symb_nt=1" \
  "libiqo_amd/variants/m1edge0.so|--option sweep=1" "libiqo_amd/variants/m1edge0.so|--option sweep=0 --option symb_nt=1" \
  "libiqo_amd/variants/m1.so|--option sweep=0" > gpurun_out/ab6.txt 2>&1 || { tail -5 gpurun_out/ab6.txt; exit 1; }
cat gpurun_out/ab6.txt
timeout -k 10 300 python scripts/ratio_sweep.py --match "x720" > gpurun_out/rs6.txt 2>&1 || { tail -5 gpurun_out/rs6.txt; exit 1; }
timeout -k 10 300 python scripts/ratio_sweep.py --match "x360" >> gpurun_out/rs6.txt 2>&1 || { tail -5 gpurun_out/rs6.txt; exit 1; }
timeout -k 10 300 python scripts/ratio_sweep.py --match "x480" >> gpurun_out/rs6.txt 2>&1 || { tail -5 gpurun_out/rs6.txt; exit 1; }
cat gpurun_out/rs6.txt
