set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_forward.py tests/test_gpu_backward.py -q > gpurun_out/t1.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t1.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --stages > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --stages --fast-exp > gpurun_out/bench_fast.log 2>&1; rc=$?; echo "bench fast rc=$rc"
exit $rc
