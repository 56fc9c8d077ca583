#!/bin/bash
# Same-box A/B of two library builds (guava_renderer_amd/lib/ab/libgsr_{a,b}.so): B's parity tests,
# then the bench alternating A and B.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abl
mkdir -p $O
GSR_LIB=$PWD/guava_renderer_amd/lib/ab/libgsr_b.so timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_fullsize.py tests/test_gpu_backward.py tests/test_gpu_deform.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest(B) rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in a b a b a b; do for acc in "" ${ABL_EXACT:-}; do
  GSR_LIB=$PWD/guava_renderer_amd/lib/ab/libgsr_$v.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --stages ${ABL_BENCH:-} $acc > $O/b.json 2>$O/b.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail $O/b.err; exit $rc; }
  python -c "import json,sys; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print('$v $acc', d['value'], s['render_fwd'], s.get('render_bwd'), s['preprocess'], s['ordered_scatter'], s['depth_sort'], s['chunk_count'], d.get('deform_ms_per_step'))"
done; done
