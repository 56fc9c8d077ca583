#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
timeout -k 10 300 python -m pytest tests/test_gpu_forward.py -x -q > gpurun_out/s/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for m in 0 1 2; do
  GSR_RENDER_SCHED=$m timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/s/bench_$m.json 2>&1; rc=$?; echo "sched $m rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.loads(open('gpurun_out/s/bench_$m.json').read().strip().splitlines()[-1]); print($m, d['value'], d['roofline']['avg_launch_ms'])"
done
