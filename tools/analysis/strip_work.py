"""Per-strip render work on one C2 frame (CPU oracle state): survivors a 16x4 strip must blend
before all its pixels finish.  The slowest strip bounds render_fwd's latency."""
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
m2 = st["means2D"].reshape(-1, 2)
co = st["conic_opacity"].reshape(-1, 4)
ranges = st["ranges"].reshape(-1, 2)
pl = st["point_list"]
fT = st["final_T"].reshape(H, W)
nc = st["n_contrib"].reshape(H, W)
gx = W // 16
work = []
for t in range(ranges.shape[0]):
    a, b = ranges[t]
    if b <= a:
        continue
    g = pl[a:b]
    tx, ty = t % gx, t // gx
    for s in range(4):
        xs = tx * 16 + np.arange(16, dtype=np.float32)
        ys = ty * 16 + s * 4 + np.arange(4, dtype=np.float32)
        X, Y = np.meshgrid(xs, ys)
        dx = m2[g, 0][:, None] - X.reshape(1, -1)
        dy = m2[g, 1][:, None] - Y.reshape(1, -1)
        power = -0.5 * (co[g, 0][:, None] * dx * dx + co[g, 2][:, None] * dy * dy) - co[g, 1][:, None] * dx * dy
        alpha = np.minimum(0.99, co[g, 3][:, None] * np.exp(power))
        ok = (power <= 0) & (alpha >= 1 / 255.0)
        # pixel stop position: terminated pixels stop right after their last contributor
        yy, xx = ys.astype(int), xs.astype(int)
        ncs = nc[np.ix_(yy, xx)].reshape(-1)
        term = (fT[np.ix_(yy, xx)].reshape(-1) * 1.0) < 1.0  # placeholder, refined below
        # a pixel terminated iff some later survivor would have pushed T below 1e-4; approximate by
        # final_T < 0.01 (opaque)  -> stop at n_contrib + 1, else list end
        opaque = fT[np.ix_(yy, xx)].reshape(-1) < 0.01
        stop = np.where(opaque, ncs + 1, b - a)
        smax = int(stop.max())
        surv = ok[:smax].any(1).sum()
        work.append((int(surv), t, s, b - a))
work.sort(reverse=True)
ws = np.array([w[0] for w in work])
print("strips", len(ws), "total survivors", ws.sum(), "mean", ws.mean().round(1))
print("top 10 (survivors, tile, strip, list len):", work[:10])
print("p50 %d p90 %d p99 %d max %d" % tuple(np.percentile(ws, [50, 90, 99, 100])))
