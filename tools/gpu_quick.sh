#!/bin/bash
# Quick GPU check: forward/backward/golden parity tests, then the bench (exact and fast exp) with
# stage timing and work counters.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/q
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/q/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/q/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --stages > gpurun_out/q/bench.json 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/q/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --fast-exp > gpurun_out/q/bench_fast.json 2>&1; rc=$?; echo "bench fast rc=$rc"; tail -1 gpurun_out/q/bench_fast.json
exit $rc
