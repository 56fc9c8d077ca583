#!/bin/bash
# Same-box A/B of render_bwd variants (lib/ab/libgsr_<v>.so): backward parity tests on each non-a
# variant, then the training bench round-robin (render_bwd / render_fwd stage times).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bab
mkdir -p $O
V=${VARIANTS:-a b}
for v in $V; do
  [ "$v" = a ] && continue
  GSR_LIB=$PWD/guava_renderer_amd/lib/ab/libgsr_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_train.py tests/test_golden.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1; rc=$?; echo "pytest($v) rc=$rc"; tail -1 $O/pytest_$v.log
  [ $rc -eq 0 ] || exit $rc
done
for r in 1 2 3; do for v in $V; do
  GSR_LIB=$PWD/guava_renderer_amd/lib/ab/libgsr_$v.so timeout -k 10 300 python bench.py --pipeline train --batch 6 --steps 50 --warmup 5 --no-cpu-baseline --stages > $O/b.json 2>$O/b.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail $O/b.err; exit $rc; }
  python -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print('$v', d['value'], s.get('render_bwd'), s.get('render_fwd'))"
done; done
