#!/bin/bash
# k_deform_gaussians timing ablations over tools/deform_only.py: frames per workgroup 1 / 4 / 8 and
# a build without the output stores (lib/ab/libgsr_ns.so, -DGSR_DEFORM_NOSTORE=1)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/dabl
mkdir -p $OUT
for v in "1 main" "4 main" "8 main" "16 main" "8 ns"; do
  set -- $v
  L=""; [ "$2" = ns ] && L=$PWD/guava_renderer_amd/lib/ab/libgsr_ns.so
  GSR_LIB=$L GSR_DEFORM_FRAMES=$1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$1$2 -o run -- python3 tools/deform_only.py 20 > $OUT/$1$2.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 $OUT/$1$2.log; exit $rc; }
  echo "== fpw=$1 lib=$2"; python3 tools/prof_db.py $OUT/$1$2/run_results.db deform_g face
done
