set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 400 python -m pytest tests/test_gpu_forward.py tests/test_gpu_backward.py -q > gpurun_out/t1.log 2>&1; rc=$?; echo "pytest rc=$rc"
ok $rc || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"
ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --stages > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"
exit $rc
