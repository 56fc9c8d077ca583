#!/bin/bash
# Counters of the training step (config 4): kernel-trace stats, two SQ passes (instruction mix,
# wait/issue cycles) and the FETCH_SIZE / WRITE_SIZE passes, each in its own rocprofv3 run.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/ptrain
mkdir -p $OUT
B="python3 bench.py --pipeline train --batch 6 --steps 3 --warmup 1 --no-cpu-baseline"
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- $B > $OUT/kt.log 2>&1; rc=$?; echo "kt rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA -d $OUT/pmc1 -o run --output-format csv -- $B > $OUT/pmc1.log 2>&1; rc=$?; echo "pmc1 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $OUT/pmc2 -o run --output-format csv -- $B > $OUT/pmc2.log 2>&1; rc=$?; echo "pmc2 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1; rc=$?; echo "write rc=$rc"
python3 tools/pmc_table.py $OUT/pmc1 $OUT/pmc2 $OUT/fetch $OUT/write > $OUT/table.txt 2>&1
exit $rc
