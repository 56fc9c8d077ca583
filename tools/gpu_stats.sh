#!/bin/bash
# Counter-test + bench with work counters + two SQ PMC passes on render_fwd.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/stats
mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_gpu_forward.py -q -k counters > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --stages --steps 10 > $OUT/bench.json 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc1.log 2>&1; rc=$?; echo "pmc1 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAIT_INST_LDS -d $OUT/pmc2 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc2.log 2>&1; rc=$?; echo "pmc2 rc=$rc"
exit $rc
