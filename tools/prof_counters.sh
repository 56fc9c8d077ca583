set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
rocprofv3 -L > gpurun_out/prof/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/kt.log 2>&1; rc=$?; echo "kt rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/prof/pmc1 -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof/pmc1.log 2>&1; rc=$?; echo "pmc1 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM -d gpurun_out/prof/pmc2 -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof/pmc2.log 2>&1; rc=$?; echo "pmc2 rc=$rc"
exit $rc
