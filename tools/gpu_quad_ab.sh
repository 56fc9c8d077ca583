#!/bin/bash
# Quad-tail A/B on one box: render tests, then the contract bench (one batch in flight, no extras)
# with GSR_QUAD_TAIL=1 / 0 / 1, each line's render_fwd launch time and work counters.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/quad_${1:-x}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_fullsize.py tests/test_gpu_api_edges.py tests/test_gpu_deform.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in 1 0 1 h; do
  H=1; Q=$v; [ $v = h ] && { H=0; Q=1; }
  GSR_HALF_TAIL=$H GSR_QUAD_TAIL=$Q timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --inflight ${INFL:-1} --steps 100 --warmup 10 > $OUT/bench_q$v.json 2> $OUT/bench_q$v.err; rc=$?
  echo "quad=$v rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench_q$v.err; exit $rc; }
  python -c "
import json; d=json.load(open('$OUT/bench_q$v.json'))
print('quad=$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['render_mfma']['useful_frac'], {k: d['render_work_per_frame'][k] for k in ('mfma_ksteps','strip_pairs_blended','half_survivors','quad_survivors') if k in d['render_work_per_frame']})"
done
for v in 1 0; do
  GSR_RENDER_QONLY=$v timeout -k 10 200 python bench.py --pipeline frame --no-cpu-baseline --no-extras --steps 8 --warmup 2 > $OUT/frame_q$v.json 2> $OUT/frame_q$v.err; rc=$?
  echo "frame qonly=$v rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/frame_q$v.err; exit $rc; }
  python -c "
import json; d=json.load(open('$OUT/frame_q$v.json'))
print('qonly=$v', d['value'], d['latency_ms_per_frame'], d['roofline']['avg_launch_ms'])"
done
