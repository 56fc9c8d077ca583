"""Where render_fwd's lane-pairs go on one C2 frame (CPU oracle state, offline).

Simulates the GPU's 8x8-strip walk: survivors = list entries that reach alpha >= 1/255 somewhere in
the strip (the exact strip test; the GPU mask is a conservative superset), taken two per k-step
until every pixel of the strip is done.  Every lane-pair of a k-step is classified as
  done      -- the pixel already stopped (T < 1e-4) or lies outside the image,
  spatial   -- alpha < 1/255 at that pixel (the Gaussian reaches only other pixels of the strip),
  useful    -- the pixel takes the Gaussian,
  padding   -- the missing second survivor of an odd last k-step.
Usage: python tools/analysis/waste_breakdown.py [quad]   (quad: also the same numbers for 4x4 units)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
from guava_renderer_amd import scenes  # noqa: E402

W = H = 512
sc = scenes.avatar_cloud(100000, seed=0)
cam = scenes.frame_cameras(1, W, H, seed=1000)[0]
oracle.set_threads(8)
_, _, _, st = oracle.forward(sc["means3D"], sc["colors"], sc["opacities"], sc["scales"], sc["rotations"], None,
                             cam["viewmatrix"], cam["projmatrix"], W, H, cam["tanfovx"], cam["tanfovy"],
                             np.zeros(32, np.float32))
m2 = st["means2D"].reshape(-1, 2).astype(np.float64)
co = st["conic_opacity"].reshape(-1, 4).astype(np.float64)
ranges = st["ranges"].reshape(-1, 2)
pl = st["point_list"]
gx = W // 16


def unit_walk(g, xs, ys):
    """k-step walk of one unit of pixels (xs, ys flattened) over list g -> counts."""
    dx = m2[g, 0][:, None] - xs[None, :]
    dy = m2[g, 1][:, None] - ys[None, :]
    power = -0.5 * (co[g, 0][:, None] * dx * dx + co[g, 2][:, None] * dy * dy) - co[g, 1][:, None] * dx * dy
    alpha = np.minimum(0.99, co[g, 3][:, None] * np.exp(power))
    alpha = np.where(power > 0, 0.0, alpha)
    ok = alpha >= 1.0 / 255.0
    surv = np.nonzero(ok.any(1))[0]
    if surv.size == 0:
        return dict(ksteps=0, done=0, spatial=0, useful=0, padding=0, surv=0)
    a = alpha[surv]
    okS = ok[surv]
    n, npx = a.shape
    T = np.ones(npx)
    done = np.zeros(npx, bool)
    c = dict(ksteps=0, done=0, spatial=0, useful=0, padding=0, surv=int(n))
    for k0 in range(0, n, 2):
        if done.all():
            break
        c["ksteps"] += 1
        for j in (k0, k0 + 1):
            if j >= n:
                c["padding"] += npx
                continue
            take = okS[j] & ~done
            testT = T * (1 - np.where(take, a[j], 0.0))
            term = take & (testT < 1e-4)
            contrib = take & ~term
            c["done"] += int(done.sum())
            c["spatial"] += int((~done & ~okS[j]).sum())
            c["useful"] += int(contrib.sum())
            c["done"] += int(term.sum())  # terminating pair: nothing added
            T = np.where(contrib, testT, T)
            done |= term
    return c


def run(unit_w, unit_h):
    tot = dict(ksteps=0, done=0, spatial=0, useful=0, padding=0, surv=0)
    per_unit = []
    for t in range(ranges.shape[0]):
        a, b = ranges[t]
        if b <= a:
            continue
        g = pl[a:b].astype(np.int64)
        tx, ty = t % gx, t // gx
        for uy in range(16 // unit_h):
            for ux in range(16 // unit_w):
                xs = tx * 16 + ux * unit_w + np.arange(unit_w, dtype=np.float64)
                ys = ty * 16 + uy * unit_h + np.arange(unit_h, dtype=np.float64)
                X, Y = np.meshgrid(xs, ys)
                c = unit_walk(g, X.ravel(), Y.ravel())
                per_unit.append(c["ksteps"])
                for k in tot:
                    tot[k] += c[k]
    lanes = tot["done"] + tot["spatial"] + tot["useful"] + tot["padding"]
    print(f"unit {unit_w}x{unit_h}: k-steps {tot['ksteps']}, survivors {tot['surv']}, lane-pairs {lanes}")
    for k in ("useful", "spatial", "done", "padding"):
        print(f"   {k:8s} {tot[k]:10d}  {tot[k] / max(lanes, 1):.3f}")
    pu = np.array(per_unit)
    print("   k-steps per unit: mean %.1f p50 %d p90 %d p99 %d max %d" %
          (pu.mean(), *np.percentile(pu, [50, 90, 99, 100])))
    return tot


run(8, 8)
if len(sys.argv) > 1 and sys.argv[1] == "quad":
    run(4, 4)
    run(8, 4)
