#!/bin/bash
# After tools/gpu_round.sh: the training line (400 steps) with its kernel-trace summary, the
# render_bwd issue counters, the per-frame drop-in line and the config-5 raster line.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT
timeout -k 10 300 python bench.py --pipeline train --batch 6 --steps 400 --warmup 20 --stages --no-cpu-baseline > $OUT/bench_train400.json 2> $OUT/bench_train400.err; rc=$?; echo "train400 rc=$rc"; tail -c 300 $OUT/bench_train400.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_train -o run --output-format csv -- python3 bench.py --pipeline train --batch 6 --no-cpu-baseline --steps 20 --warmup 3 > $OUT/kt_train.log 2>&1; rc=$?; echo "kt_train rc=$rc"
[ $rc -eq 0 ] || exit $rc
PMC_KERNEL=k_render_bwd PMC_BENCH="--pipeline train --batch 6" timeout -k 10 500 bash tools/gpu_pmc_issue.sh > $OUT/pmc_bwd.log 2>&1; rc=$?; echo "pmc_bwd rc=$rc"; tail -5 $OUT/pmc_bwd.log
[ $rc -eq 0 ] || exit $rc
cp gpurun_out/pmci/summary.json $OUT/pmc_bwd_summary.json
timeout -k 10 300 python bench.py --pipeline frame --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_frame.json 2> $OUT/bench_frame.err; rc=$?; echo "frame rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --pipeline raster --steps 20 --warmup 3 --no-cpu-baseline --stages > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?; echo "c5 rc=$rc"
exit $rc
