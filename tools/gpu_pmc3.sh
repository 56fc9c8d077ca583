#!/bin/bash
# PMC passes over a short bench: instruction mix / LDS / waits, and HBM bytes, per kernel.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmc3
mkdir -p $OUT
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $OUT/$name -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc
}
run a SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY && \
run b FETCH_SIZE GRBM_GUI_ACTIVE && \
run c WRITE_SIZE GRBM_GUI_ACTIVE
