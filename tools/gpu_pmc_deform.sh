#!/bin/bash
# Deform kernel counters: kernel trace, FETCH_SIZE, WRITE_SIZE and two SQ passes over
# tools/deform_only.py, each its own rocprofv3 run; summary -> gpurun_out/pmcd/pmc_deform.json
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmcd
mkdir -p $OUT
D="python3 tools/deform_only.py 3"
timeout -k 10 120 python3 tools/deform_only.py 50; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python3 tools/deform_only.py 20 > $OUT/kt.log 2>&1; rc=$?; echo "kt rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/prof_db.py $OUT/kt/run_results.db lbs deform splice pack face
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $D > $OUT/fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $D > $OUT/write.log 2>&1; rc=$?; echo "write rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/sq1 -o run --output-format csv -- $D > $OUT/sq1.log 2>&1; rc=$?; echo "sq1 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -d $OUT/sq2 -o run --output-format csv -- $D > $OUT/sq2.log 2>&1; rc=$?; echo "sq2 rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py $OUT/fetch $OUT/write deform 32 $OUT/pmc_deform.json $OUT/sq1 $OUT/sq2 > /dev/null; rc=$?
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/pmcd/pmc_deform.json"))
for k, v in d["kernels"].items():
    sq = v.get("sq", {})
    wc = sq.get("SQ_WAVE_CYCLES") or 1
    print(k, "fetchMB %.1f writeMB %.1f" % (v.get("fetch_bytes", 0) / 1e6, v.get("write_bytes", 0) / 1e6),
          "waves", sq.get("SQ_WAVES"), "valu", sq.get("SQ_INSTS_VALU"), "vmem", sq.get("SQ_INSTS_VMEM"),
          "busy", sq.get("SQ_BUSY_CYCLES"), "gui", sq.get("GRBM_GUI_ACTIVE"),
          "wait %.2f stall %.2f issue %.2f" % (sq.get("SQ_WAIT_ANY", 0) / wc, sq.get("SQ_WAIT_INST_ANY", 0) / wc,
                                              sq.get("SQ_ACTIVE_INST_ANY", 0) / wc))
PY
exit $rc
