#!/bin/bash
# Same-box timing A/B of library builds (tools/build_ab.py <tag> ... -> guava_renderer_amd/lib/ab/
# libgsr_<tag>.so) and environment switches on one bench pipeline, R rounds, interleaved:
#   tools/gpu_lib_ab.sh base fill4 n5w4 'env:GSR_RENDER_ABLATE=8' ...
# "base" is the tree's library; "env:VAR=VAL[,VAR=VAL]" runs the GSR_TUNING build tagged "tune"
# (python tools/build_ab.py tune) with those variables: the product library ignores them.
# PIPE (default avatar), BATCH (32), STEPS (100), R (2), TESTS (pytest files run first, optional).
# Prints frames/s, ms/step and render_fwd's isolated-pass launch time per variant.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/libab
mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 $O/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${R:-2}); do
  for V in "$@"; do
    (
      case "$V" in
        base) ;;
        env:*) export GSR_LIB=guava_renderer_amd/lib/ab/libgsr_tune.so
               for kv in $(echo "${V#env:}" | tr ',' ' '); do export "$kv"; done ;;
        *) export GSR_LIB=guava_renderer_amd/lib/ab/libgsr_$V.so ;;
      esac
      tag=$(echo "$V" | tr -c 'A-Za-z0-9_\n' '_')
      timeout -k 10 300 python bench.py --pipeline ${PIPE:-avatar} --batch ${BATCH:-32} --inflight ${INFL:-1} --no-cpu-baseline \
        --no-extras --steps ${STEPS:-100} --warmup 10 > $O/$tag.json 2> $O/$tag.err
      rc=$?
      [ $rc -eq 0 ] || { echo "$V rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
      python - "$V" "$O/$tag.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
rf = d.get("roofline", {})
rb = d.get("roofline_bwd", {})
print(f"{sys.argv[1]:36s} fps={d['value']:9.1f} ms={d['ms_per_step']:.4f} render_fwd={rf.get('avg_launch_ms')} frac={rf.get('frac')}"
      + (f" render_bwd={rb.get('avg_launch_ms')} ({rb.get('us_per_frame')} us/frame)" if rb else ""))
PY
    ) || exit $?
  done
done
