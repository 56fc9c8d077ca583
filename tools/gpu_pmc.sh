#!/bin/bash
# HBM traffic and issue counters of one bench workload, each counter group its own rocprofv3 pass:
#   tools/gpu_pmc.sh [avatar|train] [out.json]
# avatar (default): the contract line (32-frame C2 avatar batch) -> profiles/pmc_render_fwd.json;
# train: the config-4 training line (batch 6) -> profiles/pmc_train.json.  FETCH_SIZE is first
# calibrated on known byte counts (tools/micro/fetch_calib, built here if missing); the summary is
# stamped with the source hash, so bench.py only uses it for the library it was measured on.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PIPE=${1:-avatar}
if [ "$PIPE" = train ]; then
  WL="guava-avatar-synth-100k-512-train"; BATCH=6; DEF=profiles/pmc_train.json
else
  WL="guava-avatar-synth-100k-512-deform+raster"; BATCH=32; DEF=profiles/pmc_render_fwd.json
fi
DST=${2:-$DEF}
OUT=gpurun_out/pmc_$PIPE
mkdir -p $OUT
B="python3 bench.py --pipeline $PIPE --batch $BATCH --inflight 1 --no-cpu-baseline --no-extras --steps 3 --warmup 1"
if [ ! -x tools/micro/fetch_calib ]; then
  /opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 tools/micro/fetch_calib.hip -o tools/micro/fetch_calib || exit 1
fi
run() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d $OUT/$n -o run --output-format csv -- $B > $OUT/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; return $rc
}
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $OUT/calib -o run --output-format csv -- tools/micro/fetch_calib > $OUT/calib.log 2>&1; rc=$?; echo "calib rc=$rc"
[ $rc -eq 0 ] || exit $rc
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE || exit $?
python3 tools/pmc_summary.py $OUT/fetch $OUT/write "$WL" $BATCH $OUT/summary.json $OUT/sq1 $OUT/sq2 --calib $OUT/calib > /dev/null || exit 1
cp $OUT/summary.json $DST
python3 -c "import json; d=json.load(open('$DST')); print(d.get('fetch_calibration'), d.get('render_fwd_issue'), d['hbm_bytes_per_launch'])"
