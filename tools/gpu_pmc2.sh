#!/bin/bash
# Three PMC passes over a short bench (render-oriented counters).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmc2
mkdir -p $OUT
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" -d $OUT/$name -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc
}
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE && \
run b SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_SALU SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD && \
run c TA_BUSY TA_TA_BUSY TA_ADDR_STALLED_BY_TD_CYCLES TA_DATA_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE && \
run d TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY SQ_INSTS_BRANCH SQ_INSTS_SMEM
