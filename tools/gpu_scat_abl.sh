#!/bin/bash
# ordered_scatter timing ablations (GSR_SCATTER_ABLATE: 1 = no strip test, 2 = no list store)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sabl
for a in 0 1 2 3 0; do
  GSR_SCATTER_ABLATE=$a timeout -k 10 200 python bench.py --pipeline raster --steps 30 --warmup 5 --stages --no-cpu-baseline > gpurun_out/sabl/a$a.json 2> gpurun_out/sabl/a$a.err; rc=$?
  [ $rc -eq 0 ] || [ $a -ne 0 ] || { echo "abl $a rc=$rc"; tail -3 gpurun_out/sabl/a$a.err; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sabl/a$a.json').read().strip().splitlines()[-1]); print('abl $a', d['stage_ms_per_step']['ordered_scatter'])" 2>/dev/null || echo "abl $a (no result)"
done
