#!/bin/bash
# render_bwd timing ablations (GSR_BWD_ABLATE, wrong gradients by construction) on the training bench
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/babl
for a in 0 1 2 3 0; do
  GSR_BWD_ABLATE=$a timeout -k 10 200 python bench.py --pipeline train --batch 6 --steps 20 --warmup 3 --stages --no-cpu-baseline > gpurun_out/babl/a$a.json 2> gpurun_out/babl/a$a.err; rc=$?
  [ $rc -eq 0 ] || { echo "abl $a rc=$rc"; tail -3 gpurun_out/babl/a$a.err; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/babl/a$a.json').read().strip().splitlines()[-1]); print('abl $a', d['value'], d['stage_ms_per_step']['render_bwd'])"
done
