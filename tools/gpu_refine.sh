#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/refine
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_forward.py > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error" $OUT/pytest.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --refine > $OUT/bench_refine.json 2> $OUT/bench_refine.err; rc=$?; echo "refine rc=$rc"; tail -1 $OUT/bench_refine.json; tail -3 $OUT/bench_refine.err
exit $rc
