#!/bin/bash
# Round check: smoke, all -m gpu tests, the contract bench (N=1), the per-frame drop-in bench, the
# training bench, a 2-rank gloo rehearsal of the N>1 path on one GPU, fused-SSIM at the reference's
# benchmark configuration and the CPU baselines on this host.  $1 = "notests" skips the tests.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/full
mkdir -p $OUT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"
[ $rc -eq 0 ] || exit $rc
if [ "${1:-}" != "notests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $OUT/pytest_gpu.log | tail -8
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --pipeline frame --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_frame.json 2> $OUT/bench_frame.err; rc=$?; echo "frame rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --pipeline train --batch 6 --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench_train.json 2> $OUT/bench_train.err; rc=$?; echo "train rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --pipeline raster --steps 20 --warmup 3 --no-cpu-baseline --stages > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?; echo "c5 rc=$rc"
[ $rc -eq 0 ] || exit $rc
GSR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_n2.json 2> $OUT/bench_n2.err; rc=$?; echo "n2 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_ssim.py > $OUT/ssim.json 2> $OUT/ssim.err; rc=$?; echo "ssim rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/cpu_baselines.py $OUT/cpu_baselines_gpubox.json > /dev/null 2> $OUT/cpu.err; rc=$?; echo "cpu rc=$rc"
exit $rc
