#!/bin/bash
# Texture-path counters of the contract bench (TA/TD busy and stalls, L1 request latency)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmcta
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --steps 3 --warmup 1"
timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE -d $OUT/p1 -o run --output-format csv -- $B > $OUT/p1.log 2>&1; rc=$?; echo "p1 rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmcta/p1/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gsr::", "")[:40]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in ("k_render_fwd<true, false, false, 2>", "k_ordered_scatter<0>", "k_preprocess"):
    if k in acc:
        print(k, {c: round(sum(v[1:]) / max(len(v) - 1, 1)) for c, v in sorted(acc[k].items())})
PY
