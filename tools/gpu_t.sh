#!/bin/bash
# GPU check: the -m gpu tests (optionally a subset: $1 = pytest -k expression), then the training
# bench with stage timing.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/t/pytest.log 2>&1; rc=$?
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t/pytest.log 2>&1; rc=$?
fi
echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/t/pytest.log | tail -60
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --pipeline train --batch 6 --steps 20 --warmup 3 --stages --no-cpu-baseline > gpurun_out/t/train.json 2> gpurun_out/t/train.err; rc=$?; echo "train rc=$rc"; tail -1 gpurun_out/t/train.json; tail -3 gpurun_out/t/train.err
exit $rc
