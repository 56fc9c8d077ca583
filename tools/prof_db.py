"""Per-(kernel, grid) average durations from a rocprofv3 rocpd database:
    python tools/prof_db.py run_results.db [name-substring ...]"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
pats = sys.argv[2:] or [""]
d = collections.defaultdict(list)
for n, gx, gy, dur in c.execute("select name, grid_x, grid_y, duration from kernels"):
    if any(p in n for p in pats):
        d[(n.split("(")[0][-40:], gx, gy)].append(dur)
tot = 0
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v)
    print(f"{k[0]:42s} grid {k[1]:>8}x{k[2]:<4} calls {len(v):5d} avg_us {sum(v) / len(v) / 1000:9.2f}")
print("total ms", tot / 1e6)
