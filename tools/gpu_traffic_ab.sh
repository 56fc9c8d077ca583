#!/bin/bash
# Same-box HBM-traffic A/B of render_fwd (and repeatability of the counter pass), each variant its
# own FETCH_SIZE and WRITE_SIZE rocprofv3 passes over the contract workload (one batch in flight):
#   base  -- the tree's library, twice (run-to-run spread of the counters);
#   fill4 -- empty tiles as per-strip dword stores (guava_renderer_amd/lib/ab/libgsr_fill4.so,
#            built here by `python tools/build_ab.py fill4 -DGSR_FILL16=0`), the form before 4beb62b;
#   abl8  -- no empty-tile stores at all (GSR_RENDER_ABLATE=8, timing-only, wrong images);
#   qt1   -- the opt-in quad + half tails (GSR_QUAD_TAIL=1);
#   train -- the config-4 training line twice (render_bwd's counters, unchanged kernel).
# Summaries: gpurun_out/traffic/<variant>.json (tools/pmc_summary.py).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/traffic
mkdir -p $O
A="python3 bench.py --pipeline avatar --batch 32 --inflight 1 --no-cpu-baseline --no-extras --steps 3 --warmup 1"
T="python3 bench.py --pipeline train --batch 6 --inflight 1 --no-cpu-baseline --no-extras --steps 3 --warmup 1"
pass() {  # variant counter cmd...
  local v=$1 c=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc $c -d $O/$v/$c -o run --output-format csv -- "$@" > $O/$v.$c.log 2>&1
  local rc=$?; echo "$v $c rc=$rc"; return $rc
}
variant() {  # name pipeline-cmd (env already exported by the caller's subshell)
  local v=$1; shift
  pass $v FETCH_SIZE "$@" || return 1
  pass $v WRITE_SIZE "$@" || return 1
  python3 tools/pmc_summary.py $O/$v/FETCH_SIZE $O/$v/WRITE_SIZE "$v" 32 $O/$v.json > /dev/null || return 1
  python3 - $O/$v.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k in ("k_render_fwd", "k_render_fwd_ablate", "k_render_bwd", "k_ordered_scatter"):
    r = d["kernels"].get(k)
    if r:
        print(f"  {d['config']:7s} {k:18s} fetch {r['fetch_bytes']/1e6:8.1f} MB  write {r['write_bytes']/1e6:8.1f} MB  launches {r['launches']}")
PY
}
( variant base $A ) || exit 1
( export GSR_LIB=guava_renderer_amd/lib/ab/libgsr_fill4.so; variant fill4 $A ) || exit 1
( export GSR_RENDER_ABLATE=8; variant abl8 $A ) || exit 1
( export GSR_QUAD_TAIL=1; variant qt1 $A ) || exit 1
( variant base2 $A ) || exit 1
( variant train $T ) || exit 1
( variant train2 $T ) || exit 1
