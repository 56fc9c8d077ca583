"""Print per-kernel averages of rocprofv3 counter CSVs: python tools/pmc_table.py <dir>..."""
import collections
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "gsr::" not in k:
                continue
            k = k.split("(")[0].replace("void ", "").replace("gsr::", "")
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(k, {c: round(sum(x) / len(x)) for c, x in sorted(v.items())})
