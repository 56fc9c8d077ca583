#!/bin/bash
# HBM traffic of the training line's kernels (render_fwd, render_bwd, ...): one FETCH_SIZE and one
# WRITE_SIZE rocprofv3 pass over `bench.py --pipeline train --batch 6`, summarised per launch by
# tools/pmc_summary.py -> gpurun_out/ptr/pmc_train.json (copy to profiles/ for the bench line).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ptr
mkdir -p $O
B="python3 bench.py --pipeline train --batch 6 --no-cpu-baseline --steps 3 --warmup 1"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $B > $O/fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $B > $O/write.log 2>&1; rc=$?; echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py $O/fetch $O/write guava-avatar-synth-100k-512-train 6 $O/pmc_train.json
