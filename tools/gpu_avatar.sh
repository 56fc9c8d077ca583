#!/bin/bash
# Deform parity tests, then the avatar (deform + raster) bench and the raster-only bench.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/avatar
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_deform.py > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -12 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --stages > $OUT/bench_avatar.json 2> $OUT/bench_avatar.err; rc=$?; echo "avatar rc=$rc"; tail -1 $OUT/bench_avatar.json; tail -5 $OUT/bench_avatar.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --pipeline raster --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_raster.json 2>&1; rc=$?; echo "raster rc=$rc"; tail -1 $OUT/bench_raster.json
exit $rc
