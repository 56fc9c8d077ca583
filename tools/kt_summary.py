"""Per-kernel call counts and average / total durations from a rocprofv3 --kernel-trace output
directory (its SQLite database), largest total first:  python tools/kt_summary.py <dir> [--csv out.csv]"""
import csv
import glob
import sqlite3
import sys

db = sorted(glob.glob(sys.argv[1] + "/**/*.db", recursive=True))[-1]
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), avg(end - start), sum(end - start) from kernels group by name "
                 "order by sum(end - start) desc").fetchall()
if "--csv" in sys.argv:
    with open(sys.argv[sys.argv.index("--csv") + 1], "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs"])
        for n, k, a, t in rows:
            w.writerow([n, k, int(t), round(a, 1)])
for n, k, a, t in rows:
    print(f"{a / 1000:9.2f} us x {k:5d}  {n[:90]}")
