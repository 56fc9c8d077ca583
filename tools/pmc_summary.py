"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes for each kernel.

    python tools/pmc_summary.py <fetch_dir> <write_dir> <config> <batch> <out.json>

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


def main():
    fdir, wdir, config, batch, out = sys.argv[1:6]
    fetch = _per_kernel(fdir, "FETCH_SIZE")
    write = _per_kernel(wdir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        fb = 2.0 * fetch.get(k, (0.0, 0))[0]
        wb = write.get(k, (0.0, 0))[0]
        kernels[k] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
                      "launches": max(fetch.get(k, (0, 0))[1], write.get(k, (0, 0))[1])}
    rf = kernels.get("k_render_fwd", {})
    res = {"config": config, "batch": int(batch),
           "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count), WRITE_SIZE KiB x1024",
           "hbm_bytes_per_launch": rf.get("hbm_bytes"), "kernels": kernels}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
