"""Per-frame GPU timeline of the per-frame drop-in loop, from a rocprofv3 --kernel-trace CSV:
    python tools/frame_gaps.py <trace dir or kernel_trace.csv> [--marker k_render_quad] [--skip 20]
A frame is the span between the ends of two consecutive marker kernels.  For the median frame
(after `skip` frames) prints each kernel in launch order with its duration and the idle gap before
it, then the medians over all frames of: frame span, GPU busy time and idle time."""
import csv
import glob
import os
import statistics
import sys


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        path = sorted(glob.glob(path + "/**/*kernel_trace.csv", recursive=True))[-1]
    mk = sys.argv[sys.argv.index("--marker") + 1] if "--marker" in sys.argv else "k_render_quad"
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 20
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0])
                  for r in csv.DictReader(open(path)))
    ends = [i for i, r in enumerate(rows) if mk in r[2]]
    frames = []
    for a, b in zip(ends[skip:], ends[skip + 1:]):
        ks = rows[a + 1:b + 1]
        t_prev = rows[a][1]
        seq = []
        busy = 0
        for s, e, n in ks:
            seq.append((n, max(0, s - t_prev), e - s))
            busy += e - s
            t_prev = max(t_prev, e)
        frames.append((rows[b][1] - rows[a][1], busy, seq))
    if not frames:
        print("no frames")
        return
    spans = [f[0] for f in frames]
    med = statistics.median(spans)
    f = min(frames, key=lambda x: abs(x[0] - med))
    print(f"{len(frames)} frames: span median {med / 1e3:.1f} us, busy median "
          f"{statistics.median(x[1] for x in frames) / 1e3:.1f} us, idle median "
          f"{statistics.median(x[0] - x[1] for x in frames) / 1e3:.1f} us")
    print(f"{'kernel':60s} {'gap us':>8s} {'dur us':>8s}")
    for n, g, d in f[2]:
        print(f"{n[:60]:60s} {g / 1e3:8.1f} {d / 1e3:8.1f}")


if __name__ == "__main__":
    main()
