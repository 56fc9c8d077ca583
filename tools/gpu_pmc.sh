#!/bin/bash
# SQ counter passes over the bench (render_fwd and binning kernels); results in gpurun_out/pmc.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 > $OUT/kt.log 2>&1; rc=$?; echo "kt rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/p1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/p1.log 2>&1; rc=$?; echo "p1 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM -d $OUT/p2 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/p2.log 2>&1; rc=$?; echo "p2 rc=$rc"
exit $rc
