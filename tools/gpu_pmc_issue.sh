#!/bin/bash
# Issue/stall counters of one kernel (PMC_KERNEL, default k_render_fwd) of the bench (extra args in
# PMC_BENCH) and TA/TD busy, three rocprofv3 passes;
# per-launch averages (first launch dropped) -> gpurun_out/pmci/summary.json
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmci
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 ${PMC_BENCH:-}"
export PMC_KERNEL=${PMC_KERNEL:-k_render_fwd}
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/p1 -o run --output-format csv -- $B > $OUT/p1.log 2>&1; rc=$?; echo "p1 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- $B > $OUT/p2.log 2>&1; rc=$?; echo "p2 rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE -d $OUT/p3 -o run --output-format csv -- $B > $OUT/p3.log 2>&1; rc=$?; echo "p3 rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv, glob, collections, json, os
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in ("p1", "p2", "p3"):
    for f in glob.glob(f"gpurun_out/pmci/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gsr::", "")
            if os.environ["PMC_KERNEL"] not in k:
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: sum(v[1:]) / max(len(v) - 1, 1) for c, v in sorted(d.items())} for k, d in acc.items()}
json.dump(out, open("gpurun_out/pmci/summary.json", "w"), indent=1)
for k, d in out.items():
    print(k, {c: round(v) for c, v in d.items()})
PY
