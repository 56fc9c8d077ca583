#!/bin/bash
# Same-box sweep of the render placement (bench.py --cu-split K [--cu-mode M]) on the contract
# workload with 4 batches in flight, R rounds interleaved:
#   tools/gpu_split_ab.sh none 0 16 32 48 lo:32
# "none" = the shared default; K = prep slice of K CUs ("spread"); lo:K = the first K CUs;
# rs:K/P = K render streams, the batches' streams at priority P (e.g. rs:2/-1).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/split
mkdir -p $O
for r in $(seq 1 ${R:-2}); do
  for V in "$@"; do
    case "$V" in
      none) A="" ;;
      lo:*) A="--cu-split ${V#lo:} --cu-mode lo" ;;
      rs:*) K=$(echo ${V#rs:} | cut -d/ -f1); PR=$(echo ${V#rs:} | cut -s -d/ -f2)
            A="--render-streams $K --prep-priority ${PR:-0}" ;;
      *) A="--cu-split $V" ;;
    esac
    tag=$(echo "$V" | tr -c 'A-Za-z0-9_\n' '_')
    timeout -k 10 300 python bench.py --inflight ${INFL:-4} --no-cpu-baseline --no-extras --steps ${STEPS:-100} \
      --warmup 10 $A > $O/$tag.json 2> $O/$tag.err
    rc=$?
    [ $rc -eq 0 ] || { echo "$V rc=$rc"; tail -5 $O/$tag.err; exit $rc; }
    python - "$V" "$O/$tag.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
rf = d.get("roofline", {})
print(f"{sys.argv[1]:10s} fps={d['value']:9.1f} ms={d['ms_per_step']:.4f} render_fwd(isolated)={rf.get('avg_launch_ms')} "
      f"placement={d['config'].get('placement')}")
PY
  done
done
