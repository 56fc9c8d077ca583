#!/bin/bash
# Iteration check: GPU parity tests, avatar bench with stage timing, training-step bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/it2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for P in avatar raster; do
timeout -k 10 300 python bench.py --pipeline $P --steps 10 --warmup 3 --no-cpu-baseline --stages > $OUT/bench_$P.json 2>&1; rc=$?; echo "bench $P rc=$rc"
[ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.loads(open('$OUT/bench_$P.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_ms'], d.get('stage_ms_per_step'))"
done
timeout -k 10 300 python bench.py --pipeline train --batch 6 --steps 10 --warmup 3 --stages > $OUT/bench_train.json 2>&1; rc=$?; echo "train rc=$rc"
[ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.loads(open('$OUT/bench_train.json').read().strip().splitlines()[-1]); print(d['value'], d.get('stage_ms_per_step'))"
