#!/bin/bash
# split-bf16 colour accumulation: parity (tolerance) tests, then the bench with and without it.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/split
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_fullsize.py tests/test_gpu_backward.py -x -v -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for args in "" "--exact-accum" ""; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --stages $args > $O/b.json 2>$O/b.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail $O/b.err; exit $rc; }
  python -c "import json,sys; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$args', d['value'], d['roofline']['avg_launch_ms'], d['stage_ms_per_step'])"
done
