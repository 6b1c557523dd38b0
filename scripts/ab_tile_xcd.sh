timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
V=libiqo_amd/variants
STEPS=50 REPS=2 timeout -k 10 600 bash scripts/ab2.sh "$V/xcd0.so|--config g1" "$V/xcd1.so|--config g1" "$V/xcd2.so|--config g1" "$V/xcd0.so|--config g2" "$V/xcd1.so|--config g2" "$V/xcd2.so|--config g2" "$V/xcd0.so|--config g3" "$V/xcd1.so|--config g3" "$V/xcd2.so|--config g3"
