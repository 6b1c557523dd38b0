set -o pipefail
cd $GRAFT_REPO_ROOT
export IQO_REQUIRE_HIP=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt7.log 2>&1 || { tail -40 gpurun_out/pt7.log; exit 1; }
tail -2 gpurun_out/pt7.log
REPS=2 STEPS=40 BENCH_EXTRA="--no-probe --alt-frames 0 --no-verify" bash scripts/ab2.sh \
  "libiqo_amd/libiqo_hip.so|--option sweep=0" "libiqo_amd/libiqo_hip.so|--option sweep=1" \
  "libiqo_amd/libiqo_hip.so|--option sweep=1 --option sweep_wg=1" "libiqo_amd/libiqo_hip.so|--option sweep=1 --option sweep_wg=2" \
  "libiqo_amd/libiqo_hip.so|--option sweep=0 --option symb_nt=1" \
  "libiqo_amd/variants/nts0.so|--option sweep=1" "libiqo_amd/variants/ntl0.so|--option sweep=1" \
  "libiqo_amd/variants/alt1.so|--option sweep=1" > gpurun_out/ab7.txt 2>&1 || { cat gpurun_out/ab7.txt; exit 1; }
cat gpurun_out/ab7.txt
timeout -k 10 300 python scripts/ratio_sweep.py > gpurun_out/rs7.txt 2>&1 || { tail -5 gpurun_out/rs7.txt; exit 1; }
cat gpurun_out/rs7.txt
