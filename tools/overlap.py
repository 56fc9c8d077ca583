"""How batches in flight overlap on the GPU, from a rocprofv3 --kernel-trace CSV (kernel_trace.csv):
    python tools/overlap.py <trace dir or kernel_trace.csv> [--kernel k_render_fwd] [--skip-frac 0.3] [--end-frac 1]
Takes the part of the trace between skip-frac and end-frac (the timed steps after warm-up), and reports the wall
span, the time with the GPU idle, with only the render kernel running, with the render kernel and
other kernels together, and with only other kernels; plus the other kernels' busy time split into
'beside the render' and 'alone' per kernel name (largest first)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(path):
    if os.path.isdir(path):
        path = sorted(glob.glob(path + "/**/*kernel_trace.csv", recursive=True))[-1]
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     r.get("Queue_Id", ""), r.get("Stream_Id", "")))
    rows.sort()
    return rows


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def measure(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def main():
    path = sys.argv[1]
    kern = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "k_render_fwd"
    skip = float(sys.argv[sys.argv.index("--skip-frac") + 1]) if "--skip-frac" in sys.argv else 0.3
    endf = float(sys.argv[sys.argv.index("--end-frac") + 1]) if "--end-frac" in sys.argv else 1.0
    rows = load(path)
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    cut, cut1 = t0 + skip * (t1 - t0), t0 + endf * (t1 - t0)
    rows = [r for r in rows if cut <= r[0] and r[1] <= cut1]
    t0 = rows[0][0]
    t1 = max(r[1] for r in rows)
    span = t1 - t0
    rend = union([(s, e) for s, e, n, *_ in rows if kern in n])
    other = union([(s, e) for s, e, n, *_ in rows if kern not in n])
    busy = union(rend + other)
    both = intersect(rend, other)
    n_r = sum(1 for r in rows if kern in r[2])
    print(f"span {span / 1e3:.1f} us over {n_r} {kern} launches ({span / 1e3 / max(n_r, 1):.1f} us per launch)")
    print(f"  idle            {(span - measure(busy)) / 1e3:10.1f} us  {(span - measure(busy)) / span:6.1%}")
    print(f"  render only     {(measure(rend) - measure(both)) / 1e3:10.1f} us  {(measure(rend) - measure(both)) / span:6.1%}")
    print(f"  render + other  {measure(both) / 1e3:10.1f} us  {measure(both) / span:6.1%}")
    print(f"  other only      {(measure(other) - measure(both)) / 1e3:10.1f} us  {(measure(other) - measure(both)) / span:6.1%}")
    per = defaultdict(lambda: [0, 0, 0])  # name -> [calls, total ns, ns beside the render]
    for s, e, n, *_ in rows:
        if kern in n:
            continue
        k = n.split("(")[0][:60]
        per[k][0] += 1
        per[k][1] += e - s
        per[k][2] += measure(intersect([[s, e]], rend))
    print(f"{'kernel':62s} {'calls':>6s} {'us/launch':>10s} {'beside':>7s}  (per {kern} launch: us alone)")
    for k, (c, tot, bes) in sorted(per.items(), key=lambda kv: -(kv[1][1] - kv[1][2])):
        print(f"{k:62s} {c:6d} {tot / c / 1e3:10.2f} {bes / max(tot, 1):7.1%}  {(tot - bes) / max(n_r, 1) / 1e3:8.2f}")


if __name__ == "__main__":
    main()
