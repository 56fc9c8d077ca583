#!/bin/bash
# Deform kernel trace A/B: MFMA blend (default) vs the streaming VALU blend (GSR_BLEND_VALU=1)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/dab
mkdir -p $OUT
for v in mfma valu; do
  E=""; [ $v = valu ] && E=1
  GSR_BLEND_VALU=$E timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$v -o run -- python3 tools/deform_only.py 20 > $OUT/$v.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 $OUT/$v.log; exit $rc; }
  echo "== $v"; grep "deform ms" $OUT/$v.log; python3 tools/prof_db.py $OUT/$v/run_results.db lbs deform splice pack
done
