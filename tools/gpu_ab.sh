#!/bin/bash
# A/B of scheduling knobs: GPU parity tests once, then the avatar and training benches under each
# environment variant given as an argument (e.g. "GSR_XCD_MAP=0" "GSR_XCD_MAP=1").
#   tools/gpu_ab.sh [--no-tests] VAR=VAL[,VAR=VAL...] ...
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/ab
mkdir -p $OUT
if [ "${1:-}" != "--no-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
  [ $rc -eq 0 ] || exit $rc
else
  shift
fi
i=0
for V in "$@"; do
  i=$((i+1))
  for P in avatar train; do
    extra=""; [ $P = train ] && extra="--batch 6"
    env $(echo "$V" | tr ',' ' ') timeout -k 10 200 python bench.py --pipeline $P $extra --steps 10 --warmup 3 --no-cpu-baseline --stages > $OUT/v${i}_$P.json 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "$V $P rc=$rc"; tail -5 $OUT/v${i}_$P.json; exit $rc; }
    python - "$V" "$P" "$OUT/v${i}_$P.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
st = d.get("stage_ms_per_step", {})
print(f"{sys.argv[1]:28s} {sys.argv[2]:6s} fps={d['value']:9.1f} fwd={st.get('render_fwd')} bwd={st.get('render_bwd')}")
EOF
  done
done
