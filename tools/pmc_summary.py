"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes for each kernel.

    python tools/pmc_summary.py <fetch_dir> <write_dir> <config> <batch> <out.json> [sq_dir ...]
        [--calib <fetch_calib_dir>]

Optional SQ counter passes (same command) add each kernel's instruction mix and wave-cycle split
(SQ_WAVE_CYCLES = SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY, MI355X_MICROARCH.md PMC
slots); --calib points at a FETCH_SIZE pass over tools/micro/fetch_calib, whose kernels read known
byte counts with render_fwd's load shapes, so the FETCH correction used is measured, not assumed.

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM [CDNA4]): both counters are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced read, so it is doubled;
WRITE_SIZE is taken as is.  Only launches after the first (warmup) of each kernel are averaged.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def _short(name):
    m = re.search(r"gsr::(k_[a-z_0-9]+)", name)
    return m.group(1) if m else None


def _per_kernel(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
    acc = defaultdict(list)
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        k = _short(r["Kernel_Name"])
        if k:
            acc[k].append(float(r["Counter_Value"]) * 1024.0)
    return {k: (sum(v[1:]) / max(len(v) - 1, 1) if len(v) > 1 else v[0], len(v)) for k, v in acc.items()}


def _all_counters(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"])):
            k = _short(r["Kernel_Name"])
            if k:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: (sum(v[1:]) / (len(v) - 1) if len(v) > 1 else v[0]) for c, v in cs.items()} for k, cs in acc.items()}


def _calibration(d):
    """FETCH_SIZE bytes / true bytes for each fetch_calib kernel (known byte counts)."""
    truth = {"k_b32": 1 << 28, "k_b128": 1 << 30, "k_uni_b128": 1 << 28}
    got = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != "FETCH_SIZE":
                continue
            m = re.search(r"(k_uni_b128|k_b128|k_b32)", r["Kernel_Name"])
            if m:
                got[m.group(1)].append(float(r["Counter_Value"]) * 1024.0)
    return {k: round(sum(v) / len(v) / truth[k], 4) for k, v in got.items()}


def main():
    argv = sys.argv[1:]
    calib_dir = None
    if "--calib" in argv:
        i = argv.index("--calib")
        calib_dir = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    fdir, wdir, config, batch, out = argv[:5]
    sq_dirs = argv[5:]
    fetch = _per_kernel(fdir, "FETCH_SIZE")
    write = _per_kernel(wdir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        fb = 2.0 * fetch.get(k, (0.0, 0))[0]
        wb = write.get(k, (0.0, 0))[0]
        kernels[k] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
                      "launches": max(fetch.get(k, (0, 0))[1], write.get(k, (0, 0))[1])}
    for d in sq_dirs:
        for k, cs in _all_counters(d).items():
            kernels.setdefault(k, {}).setdefault("sq", {}).update({c: round(v) for c, v in cs.items()})
    rf = kernels.get("k_render_fwd", {})
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from guava_renderer_amd import build as _build  # the sources the measured library was built from
    res = {"config": config, "batch": int(batch), "source_hash": _build.source_hash(),
           "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count), WRITE_SIZE KiB x1024",
           "hbm_bytes_per_launch": rf.get("hbm_bytes"), "kernels": kernels}
    if calib_dir:
        res["fetch_calibration"] = _calibration(calib_dir)
    sq = rf.get("sq", {})
    if sq.get("SQ_WAVE_CYCLES"):
        wc = sq["SQ_WAVE_CYCLES"]
        res["render_fwd_issue"] = {
            "valu_insts": sq.get("SQ_INSTS_VALU"), "salu_insts": sq.get("SQ_INSTS_SALU"),
            "mfma_insts": sq.get("SQ_INSTS_MFMA"), "vmem_insts": sq.get("SQ_INSTS_VMEM"),
            "wave_cycles_frac": {"waiting (s_waitcnt)": round(sq.get("SQ_WAIT_ANY", 0) / wc, 3),
                                 "issue-stalled": round(sq.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
                                 "issuing": round(sq.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3),
                                 "valu issuing": round(sq.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3)}}
        if sq.get("GRBM_GUI_ACTIVE"):
            # per-SIMD pipe busy: ACTIVE_INST_* are quad-cycles summed over waves; GRBM_GUI_ACTIVE
            # sums the 8 XCDs' cycles; 256 CUs x 4 SIMDs
            kc = sq["GRBM_GUI_ACTIVE"] / 8.0
            res["render_fwd_issue"]["simd_busy_frac"] = {
                "valu": round(4.0 * sq.get("SQ_ACTIVE_INST_VALU", 0) / (1024 * kc), 3),
                "salu": round(4.0 * sq.get("SQ_ACTIVE_INST_SCA", 0) / (1024 * kc), 3),
                "lds": round(4.0 * sq.get("SQ_ACTIVE_INST_LDS", 0) / (1024 * kc), 3)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
