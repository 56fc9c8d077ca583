#!/bin/bash
# render_bwd timing ablations (GSR_BWD_ABLATE, wrong gradients) on the training bench, round-robin
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bwdabl
mkdir -p $O
for r in 1 2; do for a in 0 ${BWD_ABLS:-1 2 3 5 6}; do
  GSR_BWD_ABLATE=$a timeout -k 10 300 python bench.py --pipeline train --batch 6 --steps 50 --warmup 5 --no-cpu-baseline --stages > $O/b.json 2>$O/b.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail $O/b.err; exit $rc; }
  python -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print('abl $a', d['value'], s.get('render_bwd'), s.get('render_fwd'))"
done; done
