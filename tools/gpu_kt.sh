#!/bin/bash
# rocprofv3 kernel-trace stats of one bench configuration per argument ("base",
# "env:VAR=VAL[,VAR=VAL]" or a lib/ab tag), top kernels printed per variant:
#   ARGS="--pipeline avatar --inflight 1 --steps 50" tools/gpu_kt.sh base env:GSR_BLEND_TILED=0
#   CMD="python3 tools/frame_profile.py" O_TAG=frame tools/gpu_kt.sh base
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/kt${O_TAG:+_$O_TAG}
mkdir -p $O
for V in "$@"; do
  (
    case "$V" in
      base) ;;
      env:*) export GSR_LIB=guava_renderer_amd/lib/ab/libgsr_tune.so
             for kv in $(echo "${V#env:}" | tr ',' ' '); do export "$kv"; done ;;
      *) export GSR_LIB=guava_renderer_amd/lib/ab/libgsr_$V.so ;;
    esac
    tag=$(echo "$V" | tr -c 'A-Za-z0-9_\n' '_')
    CMD=${CMD:-python3 bench.py ${ARGS:---inflight 1 --steps 50 --warmup 5} --no-cpu-baseline --no-extras}
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- $CMD > $O/$tag.log 2>&1
    rc=$?; echo "== $V rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$tag.log; exit $rc; }
    python3 - $O/$tag <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:int(__import__("os").environ.get("TOP", "24"))]:
    print(f"  {r['Name'][:64]:66s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us {float(r['Percentage']):6.2f}%")
PY
  ) || exit $?
done
