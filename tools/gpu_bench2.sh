#!/bin/bash
# avatar + raster benches with stage timing (optionally under env variants passed as args)
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/b2
mkdir -p $OUT
for V in "${@:-X=0}"; do
for P in avatar raster; do
  env $(echo "$V" | tr ',' ' ') timeout -k 10 200 python bench.py --pipeline $P --steps 20 --warmup 5 --no-cpu-baseline --stages > $OUT/$P.json 2>&1; rc=$?
  [ $rc -eq 0 ] || { tail -5 $OUT/$P.json; exit $rc; }
  python -c "
import json; d=json.loads(open('$OUT/$P.json').read().strip().splitlines()[-1]); print('$V $P', d['value'], d['stage_ms_per_step'])"
done
done
