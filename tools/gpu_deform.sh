#!/bin/bash
# Deform check: the deform -m gpu tests, the contract bench (deform_ms_per_step) and a kernel-trace
# summary of a short bench run.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/deform
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_deform.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err; rc=$?
echo "bench rc=$rc"; python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d.get('deform_ms_per_step'))"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1; rc=$?
echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python $GRAFT_REPO_ROOT/tools/prof_db.py $GRAFT_REPO_ROOT/$OUT/prof/run_results.db lbs deform splice pack face
if [ -n "${1:-}" ]; then
  GSR_DEFORM_FRAMES=$1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof2 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof2.log 2>&1; rc=$?
  echo "prof2 (GSR_DEFORM_FRAMES=$1) rc=$rc"
  python $GRAFT_REPO_ROOT/tools/prof_db.py $GRAFT_REPO_ROOT/$OUT/prof2/run_results.db deform face
fi
exit $rc
