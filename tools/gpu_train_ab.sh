#!/bin/bash
# Training-step A/B: frame-reduced shared backward (default) vs per-frame gradients + torch sum
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/tab
mkdir -p $OUT
for v in shared perframe shared perframe; do
  E=""; [ $v = perframe ] && E=1
  GSR_TRAIN_PERFRAME=$E timeout -k 10 300 python bench.py --pipeline train --batch 6 --steps 100 --warmup 10 --stages --no-cpu-baseline > $OUT/$v.json 2> $OUT/$v.err; rc=$?
  [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 $OUT/$v.err; exit $rc; }
  python -c "import json; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print('$v', d['value'], d['ms_per_step'], 'fwd', s['render_fwd'], 'bwd', s['render_bwd'], 'pbwd', s['preprocess_bwd'])"
done
