#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/v
for m in ${VARIANTS:-0 1 2 3}; do
  GSR_RENDER_VARIANT=$m timeout -k 10 200 python -m pytest tests/test_gpu_forward.py -x -q -k "bit_exact" > gpurun_out/v/pytest_$m.log 2>&1; rc=$?; echo "variant $m pytest rc=$rc"; tail -1 gpurun_out/v/pytest_$m.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  for e in "" "--fast-exp"; do
    GSR_RENDER_VARIANT=$m timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $e > gpurun_out/v/bench_$m$e.json 2>&1; rc=$?
    [ $rc -eq 0 ] || exit $rc
    python -c "import json; d=json.loads(open('gpurun_out/v/bench_$m$e.json').read().strip().splitlines()[-1]); print('variant $m $e', d['value'], d['roofline']['avg_launch_ms'])"
  done
done
