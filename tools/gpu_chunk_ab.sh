#!/bin/bash
# ordered_scatter / count-table row size sweep (GSR_CHUNK_PASSES x 256 Gaussians per row)
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/chunk
mkdir -p $OUT
for v in 1 4 16 1 4 16; do
  GSR_CHUNK_PASSES=$v timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --stages > $OUT/b$v.json 2> $OUT/b$v.err; rc=$?
  [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 $OUT/b$v.err; exit $rc; }
  python -c "import json; d=json.loads(open('$OUT/b$v.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print('passes=$v', d['value'], d['ms_per_step'], {k: s[k] for k in ('chunk_count','tile_scan','ordered_scatter','render_fwd')})"
done
GSR_CHUNK_PASSES=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; echo "pytest(16) rc=$?"; tail -2 $OUT/pytest.log
