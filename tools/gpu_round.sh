#!/bin/bash
# Full GPU pass: parity tests, the contract bench (with cpu_baseline), a kernel-trace/stats profile of
# the bench, separate FETCH_SIZE / WRITE_SIZE PMC passes (HBM traffic of render_fwd), and the
# training-step bench (config 4).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT
WL="guava-avatar-synth-100k-512-deform+raster"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_write.log 2>&1; rc=$?; echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
python tools/pmc_summary.py $OUT/pmc_fetch $OUT/pmc_write "$WL" 32 $OUT/pmc_render_fwd.json > /dev/null && cp $OUT/pmc_render_fwd.json profiles/pmc_render_fwd.json
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --stages --steps 10 > $OUT/bench_stages.json 2>&1; rc=$?; echo "stages rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 > $OUT/kt.log 2>&1; rc=$?; echo "kt rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --pipeline train --batch 6 --steps 10 --warmup 3 --stages > $OUT/bench_train.json 2> $OUT/bench_train.err; rc=$?; echo "train rc=$rc"; tail -1 $OUT/bench_train.json
exit $rc
