#!/bin/bash
# render_fwd counters for the bench line: FETCH_SIZE calibration on known byte counts
# (tools/micro/fetch_calib), then FETCH_SIZE, WRITE_SIZE and two SQ passes over the contract bench,
# each its own rocprofv3 run; summary -> profiles/pmc_render_fwd.json (read by bench.py).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmcf
mkdir -p $OUT
WL="guava-avatar-synth-100k-512-deform+raster"
B="python3 bench.py --no-cpu-baseline --steps 3 --warmup 1"
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $OUT/calib -o run --output-format csv -- tools/micro/fetch_calib > $OUT/calib.log 2>&1; rc=$?; echo "calib rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1; rc=$?; echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/sq1 -o run --output-format csv -- $B > $OUT/sq1.log 2>&1; rc=$?; echo "sq1 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -d $OUT/sq2 -o run --output-format csv -- $B > $OUT/sq2.log 2>&1; rc=$?; echo "sq2 rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py $OUT/fetch $OUT/write "$WL" 32 $OUT/pmc_render_fwd.json $OUT/sq1 $OUT/sq2 --calib $OUT/calib > /dev/null && cp $OUT/pmc_render_fwd.json profiles/pmc_render_fwd.json; rc=$?
python3 -c "import json; d=json.load(open('$OUT/pmc_render_fwd.json')); print(d.get('fetch_calibration'), d.get('render_fwd_issue'), d['hbm_bytes_per_launch'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 100 --warmup 10 > $OUT/kt.log 2>&1; rc=$?; echo "kt rc=$rc"
exit $rc
