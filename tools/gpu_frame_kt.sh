#!/bin/bash
# rocprofv3 kernel trace of the per-frame drop-in path (tools/frame_profile.py) per library variant
# ("base", "env:VAR=VAL[,VAR=VAL]" on the tuning build, or a tag of
# guava_renderer_amd/lib/ab/libgsr_<tag>.so); per-kernel averages into
# gpurun_out/frame_kt/<tag>.txt (tools/kt_summary.py).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/frame_kt
mkdir -p $O
for V in "$@"; do
  tag=$(echo "$V" | tr -c 'A-Za-z0-9_\n' '_')
  (
    case "$V" in
      base) unset GSR_LIB ;;
      env:*) export GSR_LIB=guava_renderer_amd/lib/ab/libgsr_tune.so
             for kv in $(echo "${V#env:}" | tr ',' ' '); do export "$kv"; done ;;
      *) export GSR_LIB=guava_renderer_amd/lib/ab/libgsr_$V.so ;;
    esac
    timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$tag -o run -- python3 tools/frame_profile.py > $O/$tag.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "$V rc=$rc"; tail -5 $O/$tag.log; exit $rc; }
    python3 tools/kt_summary.py $O/$tag > $O/$tag.txt && echo "== $V" && head -${KT_TOP:-12} $O/$tag.txt && grep "ms/frame" $O/$tag.log
  ) || exit $?
done
