#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/bwd
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_backward.py tests/test_golden.py -m gpu > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" $OUT/pytest.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --pipeline train --batch 6 --steps 10 --warmup 3 --stages > $OUT/bench_train.json 2> $OUT/bench_train.err; rc=$?; echo "train rc=$rc"; tail -1 $OUT/bench_train.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
exit $rc
