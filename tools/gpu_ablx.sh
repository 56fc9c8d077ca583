#!/bin/bash
# Same-box A/B/C/... of library builds guava_renderer_amd/lib/ab/libgsr_<v>.so for v in $VARIANTS
# (default "a b"); variant v may carry extra environment in ENV_<v> ("K=V K2=V2").  Parity tests
# of every variant but a, then the bench round-robin.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abl
mkdir -p $O
V=${VARIANTS:-a b}
for v in $V; do
  [ "$v" = a ] && continue
  e=ENV_$v; env ${!e:-} GSR_LIB=$PWD/guava_renderer_amd/lib/ab/libgsr_$v.so timeout -k 10 600 python -u -m pytest ${ABL_TESTS:-tests/test_gpu_forward.py tests/test_gpu_fullsize.py} -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1; rc=$?; echo "pytest($v) rc=$rc"; tail -1 $O/pytest_$v.log
  [ $rc -eq 0 ] || exit $rc
done
for r in 1 2 3; do for v in $V; do
  e=ENV_$v
  env ${!e:-} GSR_LIB=$PWD/guava_renderer_amd/lib/ab/libgsr_$v.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --stages ${ABL_BENCH:-} > $O/b.json 2>$O/b.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail $O/b.err; exit $rc; }
  python -c "import json,sys; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print('$v', d['value'], s['render_fwd'], s['preprocess'], s['ordered_scatter'])"
done; done
