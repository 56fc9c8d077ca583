#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pr
for m in 0 256 1024 4096 16384; do
  GSR_PRIO_ITEMS=$m timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/pr/bench_$m.json 2>&1; rc=$?
  [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.loads(open('gpurun_out/pr/bench_$m.json').read().strip().splitlines()[-1]); print('prio $m', d['value'], d['roofline']['avg_launch_ms'])"
done
