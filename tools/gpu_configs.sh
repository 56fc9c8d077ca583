#!/bin/bash
# Secondary bench lines: raster-only C2, C5 raster, two batches in flight, refiner epilogue.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cfg
mkdir -p $O
for args in "--pipeline raster" "--pipeline raster --config c5" "--inflight 2" "--refine"; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --stages $args > $O/b.json 2>$O/b.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench rc=$rc ($args)"; tail $O/b.err; exit $rc; }
  tail -1 $O/b.json > "$O/$(echo $args | tr ' -' '__').json"
  python -c "import json,sys; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$args', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d.get('stage_ms_per_step'))"
done
