# Round 5: steady-state band sweep of the block-shared Lanczos streamer over its shapes (C2 at 1024 and 256
# frames, Lanczos-2/4/5 4K 2:1, Lanczos-3 1080p -> 540p, C1), then the full GPU suite and the host-path probes.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $ROOT
SA="timeout -k 10 150 python3 scripts/probes/steady_ab.py --settle-ms 150 --reps 6"
$SA --config c2 --frames 1024 --tag c2f1024 --arm base: --arm b64:bands=64 --arm b78:bands=78 --arm b90:bands=90 --arm b99:bands=99 --arm b108:bands=108 --arm b120:bands=120 >> $OUT/r5sa_bands2.jsonl 2>> $OUT/r5sa4.err || exit 1
$SA --config c2 --frames 256 --tag c2f256 --arm base: --arm b78:bands=78 --arm b90:bands=90 --arm b108:bands=108 --arm b120:bands=120 >> $OUT/r5sa_bands2.jsonl 2>> $OUT/r5sa4.err || exit 1
$SA --config h3 --tag h3 --arm base: --arm b64:bands=64 --arm b90:bands=90 --arm b120:bands=120 >> $OUT/r5sa_bands2.jsonl 2>> $OUT/r5sa4.err || exit 1
$SA --config h3 --frames 256 --tag h3f256 --arm base: --arm b64:bands=64 --arm b90:bands=90 --arm b120:bands=120 >> $OUT/r5sa_bands2.jsonl 2>> $OUT/r5sa4.err || exit 1
$SA --config c1 --tag c1 --arm base: --arm b10:bands=10 --arm b20:bands=20 --arm b30:bands=30 --arm s0:stack=0 --arm s2:stack=2 >> $OUT/r5sa_bands2.jsonl 2>> $OUT/r5sa4.err || exit 1
$SA --config n2 --tag n2 --arm base: --arm b15:bands=15 --arm b30:bands=30 >> $OUT/r5sa_bands2.jsonl 2>> $OUT/r5sa4.err || exit 1
timeout -k 10 200 python3 scripts/ratio_sweep.py --match "x1080->960x540" > $OUT/r5_sweep_b1.txt 2>> $OUT/r5sa4.err || exit 1
timeout -k 10 200 python3 scripts/ratio_sweep.py --match "x1080->960x540" --opt bands=45 >> $OUT/r5_sweep_b1.txt 2>> $OUT/r5sa4.err || exit 1
timeout -k 10 200 python3 scripts/ratio_sweep.py --match "x2160->1920x1080" --opt bands=90 >> $OUT/r5_sweep_b1.txt 2>> $OUT/r5sa4.err || exit 1
timeout -k 10 200 python3 scripts/ratio_sweep.py --match "lanczos:3840x2160->1920x1080" >> $OUT/r5_sweep_b1.txt 2>> $OUT/r5sa4.err || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/r5_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/r5_pytest_gpu.log; exit 1; }
tail -1 $OUT/r5_pytest_gpu.log
bash scripts/gpu_ci.sh reftool hostlat || exit 1
echo done
