#!/bin/bash
# Same-box A/B of environment variants on one bench pipeline, after the named GPU tests:
#   TESTS="tests/test_gpu_backward.py" PIPE="train --batch 6" tools/gpu_env_ab.sh VAR=VAL[,VAR=VAL] ...
# prints value and the render_fwd / render_bwd / scatter stage times per variant, 3 rounds.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/eab
mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $O/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2 3; do
  i=0
  for V in "$@"; do
    i=$((i+1))
    env $(echo "$V" | tr ',' ' ') timeout -k 10 300 python bench.py --pipeline ${PIPE:-avatar} --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --stages > $O/v$i.json 2> $O/v$i.err; rc=$?
    [ $rc -eq 0 ] || { echo "$V rc=$rc"; tail -5 $O/v$i.err; exit $rc; }
    python - "$V" "$O/v$i.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
st = d.get("stage_ms_per_step", {})
print(f"{sys.argv[1]:34s} fps={d['value']:9.1f} ms={d['ms_per_step']:.4f} fwd={st.get('render_fwd')} bwd={st.get('render_bwd')} scat={st.get('ordered_scatter')}")
PY
  done
done
