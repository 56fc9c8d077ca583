#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ns
for m in 1 2; do
  GSR_RENDER_NS=$m timeout -k 10 200 python -m pytest tests/test_gpu_forward.py tests/test_golden.py -x -q -m gpu > gpurun_out/ns/pytest_$m.log 2>&1; rc=$?; echo "ns $m pytest rc=$rc"; tail -1 gpurun_out/ns/pytest_$m.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  for e in "" "--fast-exp"; do
    GSR_RENDER_NS=$m timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $e > gpurun_out/ns/bench_$m$e.json 2>&1; rc=$?
    [ $rc -eq 0 ] || exit $rc
    python -c "import json; d=json.loads(open('gpurun_out/ns/bench_$m$e.json').read().strip().splitlines()[-1]); print('ns $m $e', d['value'], d['roofline']['avg_launch_ms'], d['render_work_per_frame']['mfma_ksteps'])"
  done
done
