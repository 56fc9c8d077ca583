#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE PMC passes) of the avatar bench under an env variant ($1).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/traffic_${2:-x}
mkdir -p $OUT
env $(echo "${1:-X=0}" | tr ',' ' ') timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/f -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/f.log 2>&1 || exit 1
env $(echo "${1:-X=0}" | tr ',' ' ') timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/w -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/w.log 2>&1 || exit 1
python tools/pmc_summary.py $OUT/f $OUT/w "guava-avatar-synth-100k-512-deform+raster" 32 $OUT/pmc.json > /dev/null
python -c "
import json; d=json.load(open('$OUT/pmc.json'))
for k in ('k_render_fwd','k_ordered_scatter'):
    v=d['kernels'].get(k); print('$1', k, round(v['fetch_bytes']/1e9,3), round(v['write_bytes']/1e9,3)) if v else None"
