#!/bin/bash
# Same-box A/B of the per-frame drop-in path (bench --pipeline frame) over library variants
# guava_renderer_amd/lib/ab/libgsr_<v>.so (ENV_<v>: extra environment); forward tests on each non-a
# variant first.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fab
mkdir -p $O
V=${VARIANTS:-a b}
for v in $V; do
  [ "$v" = a ] && continue
  e=ENV_$v; env ${!e:-} GSR_LIB=$PWD/guava_renderer_amd/lib/ab/libgsr_$v.so timeout -k 10 600 python -u -m pytest ${ABL_TESTS:-tests/test_gpu_forward.py tests/test_gpu_api_edges.py} -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1; rc=$?; echo "pytest($v) rc=$rc"; tail -1 $O/pytest_$v.log
  [ $rc -eq 0 ] || exit $rc
done
for r in 1 2 3; do for v in $V; do
  e=ENV_$v
  env ${!e:-} GSR_LIB=$PWD/guava_renderer_amd/lib/ab/libgsr_$v.so timeout -k 10 300 python bench.py --pipeline frame --steps 20 --warmup 3 --no-cpu-baseline > $O/b.json 2>$O/b.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail $O/b.err; exit $rc; }
  python -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done; done
