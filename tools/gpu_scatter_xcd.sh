#!/bin/bash
# ordered_scatter chunk order A/B (GSR_SCATTER_XCD=0/1): list parity tests, avatar bench stage
# times, and one FETCH_SIZE and one WRITE_SIZE pass per variant (k_ordered_scatter traffic).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/sx
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_fullsize.py tests/test_golden.py tests/test_gpu_api_edges.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
PIPE=avatar bash tools/gpu_env_ab.sh GSR_SCATTER_XCD=0 GSR_SCATTER_XCD=1 || exit 1
for v in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    GSR_SCATTER_XCD=$v timeout -s KILL 120 rocprofv3 --pmc $c -d $O/p_${v}_$c -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/p_${v}_$c.log 2>&1; rc=$?; echo "pmc $v $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
