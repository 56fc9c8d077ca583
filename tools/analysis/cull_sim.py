"""Offline estimate of per-strip survivors for different cull tests and strip shapes (one C2
frame, CPU oracle state).  Ignores early termination (counts are upper bounds for all variants)."""
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
_, _, _, st = oracle.forward(sc["means2D"] if False else sc["means3D"], sc["colors"], sc["opacities"], sc["scales"],
                             sc["rotations"], None, cam["viewmatrix"], cam["projmatrix"], W, H,
                             cam["tanfovx"], cam["tanfovy"], np.zeros(32, np.float32))
m2 = st["means2D"].reshape(-1, 2)
co = st["conic_opacity"].reshape(-1, 4)
ranges = st["ranges"].reshape(-1, 2)
pl = st["point_list"]
gx = W // 16
thr = 1.0 / 255.0


def strips(sw, sh):
    return [(x0, y0) for y0 in range(0, 16, sh) for x0 in range(0, 16, sw)]


def count(sw, sh):
    tot_exact = 0
    tot_pix = 0
    for t in range(ranges.shape[0]):
        a, b = ranges[t]
        if b <= a:
            continue
        g = pl[a:b]
        tx, ty = t % gx, t // gx
        for (x0, y0) in strips(sw, sh):
            xs = tx * 16 + x0 + np.arange(sw, dtype=np.float32)
            ys = ty * 16 + y0 + np.arange(sh, dtype=np.float32)
            X, Y = np.meshgrid(xs, ys)
            dx = m2[g, 0][:, None] - X.reshape(1, -1)
            dy = m2[g, 1][:, None] - Y.reshape(1, -1)
            power = -0.5 * (co[g, 0][:, None] * dx * dx + co[g, 2][:, None] * dy * dy) - co[g, 1][:, None] * dx * dy
            alpha = np.minimum(0.99, co[g, 3][:, None] * np.exp(power))
            ok = (power <= 0) & (alpha >= thr)
            tot_exact += int(ok.any(1).sum())
            tot_pix += int(ok.sum())
    return tot_exact, tot_pix


print("R", st["R"])
for sw, sh in [(16, 4), (8, 8), (16, 2), (8, 4), (4, 4)]:
    e, p = count(sw, sh)
    print(f"strip {sw}x{sh}: exact-cull survivors {e}  pixel pairs alpha>=1/255 {p}  "
          f"useful frac {p / (e * sw * sh):.3f}  blended pixel-pairs {e * sw * sh}")


def box_count(sw, sh):
    a, b, c, o = co[:, 0], co[:, 1], co[:, 2], co[:, 3]
    det = a * c - b * b
    k = 2 * np.log(np.maximum(255 * o, 1e-30))
    ex = np.sqrt(np.maximum(k * c / det, 0)) * 1.05 + 1
    ey = np.sqrt(np.maximum(k * a / det, 0)) * 1.05 + 1
    tot = 0
    for t in range(ranges.shape[0]):
        r0, r1 = ranges[t]
        if r1 <= r0:
            continue
        g = pl[r0:r1]
        tx, ty = t % gx, t // gx
        for (x0, y0) in strips(sw, sh):
            sx0, sy0 = tx * 16 + x0, ty * 16 + y0
            keep = (m2[g, 0] + ex[g] >= sx0) & (m2[g, 0] - ex[g] <= sx0 + sw - 1) & \
                   (m2[g, 1] + ey[g] >= sy0) & (m2[g, 1] - ey[g] <= sy0 + sh - 1) & (o[g] >= thr)
            tot += int(keep.sum())
    return tot


for sw, sh in [(16, 4), (8, 8), (8, 4)]:
    print(f"box {sw}x{sh}: survivors {box_count(sw, sh)}")
