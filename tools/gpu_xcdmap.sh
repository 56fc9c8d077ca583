#!/bin/bash
# Render work-queue map A/B (GSR_XCD_MAP=1 tile-affine, 2 block-affine): GPU parity tests under
# map 2, avatar and training bench stage times, and an L2 hit/miss PMC pass per map.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/xm
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
PIPE=avatar bash tools/gpu_env_ab.sh GSR_XCD_MAP=1 GSR_XCD_MAP=2 || exit 1
PIPE="train --batch 6" STEPS=100 bash tools/gpu_env_ab.sh GSR_XCD_MAP=1 GSR_XCD_MAP=2 || exit 1
for v in 1 2; do
  GSR_XCD_MAP=$v timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/l2_$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/l2_$v.log 2>&1; rc=$?; echo "l2 $v rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
