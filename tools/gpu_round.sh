#!/bin/bash
# Full GPU pass: smoke, the -m gpu parity tests, the contract bench (default flags, as the driver
# runs it), a rocprofv3 kernel-trace/stats profile of the bench, and the training line.
#   tools/gpu_round.sh [tag]     (outputs under gpurun_out/round_<tag>/)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/round_${1:-x}
mkdir -p $OUT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json
[ $rc -eq 0 ] || { tail -20 $OUT/bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --inflight 1 --no-cpu-baseline --no-extras --steps 100 --warmup 10 > $OUT/kt.log 2>&1; rc=$?; echo "kt rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --pipeline train --steps 200 --warmup 10 > $OUT/bench_train.json 2> $OUT/bench_train.err; rc=$?; echo "train rc=$rc"; tail -1 $OUT/bench_train.json
exit $rc
