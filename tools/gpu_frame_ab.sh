#!/bin/bash
# Per-frame drop-in path (tools/frame_profile.py: deform B=1, GaussianRasterizer_32 B=1, both) under
# environment variants ("base" or "env:VAR=VAL[,VAR=VAL]"), R rounds interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/frameab
mkdir -p $O
for r in $(seq 1 ${R:-2}); do
  for V in "$@"; do
    (
      case "$V" in
        base) ;;
        env:*) export GSR_LIB=guava_renderer_amd/lib/ab/libgsr_tune.so  # (the product library ignores them)
               for kv in $(echo "${V#env:}" | tr ',' ' '); do export "$kv"; done ;;
        *) export GSR_LIB=guava_renderer_amd/lib/ab/libgsr_$V.so ;;
      esac
      tag=$(echo "$V" | tr -c 'A-Za-z0-9_\n' '_')
      timeout -k 10 200 python3 tools/frame_profile.py > $O/$tag.log 2>&1; rc=$?
      [ $rc -eq 0 ] || { echo "$V rc=$rc"; tail -5 $O/$tag.log; exit $rc; }
      echo "== $V"; grep "ms/frame" $O/$tag.log
    ) || exit $?
  done
done
