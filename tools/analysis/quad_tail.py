"""Longest serial chains of one C2 frame (the per-frame drop-in render is set by them): list
entries a work item walks before all its pixels finish, per 8x8 strip, 8x4 half strip and 4x4 quad,
with each unit's exact cull (alpha >= 1/255 somewhere in it).  python tools/analysis/quad_tail.py"""
import os, sys
import numpy as np
ROOT = "/root/repo"
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle
from guava_renderer_amd import scenes
W = H = 512
sc = scenes.avatar_cloud(100000, seed=0)
cam = scenes.frame_cameras(2, W, H, seed=1000)[1]
oracle.set_threads(8)
_, _, _, st = oracle.forward(sc["means3D"], sc["colors"], sc["opacities"], sc["scales"], sc["rotations"], None,
                             cam["viewmatrix"], cam["projmatrix"], W, H, cam["tanfovx"], cam["tanfovy"],
                             np.zeros(32, np.float32))
m2 = st["means2D"].reshape(-1, 2); co = st["conic_opacity"].reshape(-1, 4)
ranges = st["ranges"].reshape(-1, 2); pl = st["point_list"]; nc = st["n_contrib"].reshape(H, W)
fT = st["final_T"].reshape(H, W)
gx = W // 16
ys, xs = np.mgrid[0:16, 0:16]
res = {"strip": [], "half": [], "quad": []}
units = {"strip": [(sx, sy, 8, 8) for sy in (0, 8) for sx in (0, 8)],
         "half": [(sx, sy, 8, 4) for sy in (0, 4, 8, 12) for sx in (0, 8)],
         "quad": [(sx, sy, 4, 4) for sy in (0, 4, 8, 12) for sx in (0, 4, 8, 12)]}
for t in range(ranges.shape[0]):
    a, b = ranges[t]
    if b <= a: continue
    tx, ty = t % gx, t // gx
    g = pl[a:b]; n = b - a; pos = np.arange(1, n + 1)
    px = (tx * 16 + xs).ravel().astype(np.float32); py = (ty * 16 + ys).ravel().astype(np.float32)
    dx = m2[g, 0][:, None] - px[None]; dy = m2[g, 1][:, None] - py[None]
    c = co[g]
    power = -0.5 * (c[:, 0:1] * dx * dx + c[:, 2:3] * dy * dy) - c[:, 1:2] * dx * dy
    alpha = np.minimum(0.99, c[:, 3:4] * np.exp(power))
    reach = ((power <= 0) & (alpha >= 1/255)).reshape(n, 16, 16)
    ncp = nc[ty*16:ty*16+16, tx*16:tx*16+16]
    ft = fT[ty*16:ty*16+16, tx*16:tx*16+16]
    for kind, us in units.items():
        for (sx, sy, w, h) in us:
            r = reach[:, sy:sy+h, sx:sx+w].reshape(n, -1).any(1)
            sub_nc = ncp[sy:sy+h, sx:sx+w]; sub_ft = ft[sy:sy+h, sx:sx+w]
            end = int(sub_nc.max()) + 1 if (sub_ft < 2e-4).all() else n  # all pixels terminated -> stop
            res[kind].append(int((r & (pos <= end)).sum()))
for kind, v in res.items():
    v = np.array(v)
    print(f"{kind:6s} units {len(v):6d} survivors total {v.sum():8d} mean {v.mean():7.1f} p99 {np.percentile(v,99):7.1f} max {v.max()}")
