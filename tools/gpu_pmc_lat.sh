#!/bin/bash
# Where render_fwd's waves wait: memory latency and texture-path counters of the contract workload
# (one batch in flight), each group its own rocprofv3 pass; summary per kernel in
# gpurun_out/pmclat/summary.json and printed.  LIB=<tag> runs guava_renderer_amd/lib/ab/libgsr_<tag>.so.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/pmclat${LIB:+_$LIB}
mkdir -p $O
[ -n "${LIB:-}" ] && export GSR_LIB=guava_renderer_amd/lib/ab/libgsr_$LIB.so
B="python3 bench.py --pipeline ${PIPE:-avatar} --batch ${BATCH:-32} --inflight 1 --no-cpu-baseline --no-extras --steps 3 --warmup 1"
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d $O/$n -o run --output-format csv -- $B > $O/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; return $rc
}
run lat1 TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCP_LATENCY_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE || exit 1
run lat2 SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit 1
run lat3 TCC_HIT_sum TCC_MISS_sum SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU || exit 1
python3 - $O <<'PY'
import csv, glob, json, re, sys
from collections import defaultdict
o = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(o + "/**/*counter_collection.csv", recursive=True):
    for r in sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"])):
        m = re.search(r"gsr::(k_[a-z_0-9]+)", r["Kernel_Name"])
        if m:
            acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: {c: (sum(v[1:]) / (len(v) - 1) if len(v) > 1 else v[0]) for c, v in cs.items()} for k, cs in acc.items()}
json.dump(res, open(o + "/summary.json", "w"), indent=1)
import os
for k in os.environ.get("KERNELS", "k_render_fwd k_ordered_scatter k_chunk_count").split():
    c = res.get(k)
    if not c:
        continue
    g = lambda n: c.get(n, 0.0)
    out = {
        "l1_to_l2_read_latency_cyc": g("TCP_TCC_READ_REQ_LATENCY_sum") / max(g("TCP_TCC_READ_REQ_sum"), 1),
        "vmem_inst_latency": g("SQ_INST_LEVEL_VMEM") / max(g("SQ_INSTS_VMEM"), 1),
        "lds_inst_latency": g("SQ_INST_LEVEL_LDS") / max(g("SQ_INSTS_LDS"), 1),
        "l2_hit": g("TCC_HIT_sum") / max(g("TCC_HIT_sum") + g("TCC_MISS_sum"), 1),
        "ta_busy": g("TA_TA_BUSY_sum") / max(g("GRBM_GUI_ACTIVE"), 1) / 32.0,
        "td_busy": g("TD_TD_BUSY_sum") / max(g("GRBM_GUI_ACTIVE"), 1) / 32.0,
        "wait_lds_frac": g("SQ_WAIT_INST_LDS") / max(g("SQ_WAVE_CYCLES"), 1),
        "wait_any_frac": g("SQ_WAIT_ANY") / max(g("SQ_WAVE_CYCLES"), 1),
        "lds_bank_conflict_per_lds_inst": g("SQ_LDS_BANK_CONFLICT") / max(g("SQ_INSTS_LDS"), 1),
        "valu_insts": g("SQ_INSTS_VALU"), "salu_insts": g("SQ_INSTS_SALU"), "vmem_insts": g("SQ_INSTS_VMEM"),
        "active_valu_per_wave_cycle": g("SQ_ACTIVE_INST_VALU") / max(g("SQ_WAVE_CYCLES"), 1),
        "busy_cycles": g("SQ_BUSY_CYCLES"),
    }
    print(k, {a: round(b, 3) for a, b in out.items()})
PY
