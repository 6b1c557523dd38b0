set -o pipefail
cd $GRAFT_REPO_ROOT
export IQO_REQUIRE_HIP=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "stream_variants or device_batch or 256_frame or checkerboard or flat_frames or row_band or yuv420_planes or native_library" > gpurun_out/pt5.log 2>&1 || { tail -30 gpurun_out/pt5.log; exit 1; }
tail -2 gpurun_out/pt5.log
for o in "sweep=0" "sweep=1" "sweep_wg=1" "sweep_wg=2" "sweep=1 --option bands=24" "sweep=1 --option bands=48"; do
  timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu --no-probe --alt-frames 0 --option $o > gpurun_out/b5.log 2>&1 || { tail -5 gpurun_out/b5.log; exit 1; }
  echo "$o $(tail -1 gpurun_out/b5.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms_per_launch"], d["roofline"]["frac"], d["parity"])')"
done
