"""Where the per-frame drop-in path (GUAVA's gaussian_render.py:37-67 loop) spends host time: the
camera-field int()/float() reads of device tensors (each a device sync), the rasterizer call itself
(Python + _C + kernel launches), and the GPU time per frame (events).  Config 2, 32 frames."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diff_gaussian_rasterization_32 import GaussianRasterizationSettings, GaussianRasterizer_32  # noqa: E402
from guava_renderer_amd import scenes  # noqa: E402

dev = torch.device("cuda:0")
B, P, W = 32, 100000, 512
sc = scenes.avatar_cloud(P, seed=0)
cams = scenes.frame_cameras(B, W, W, seed=1000)
t = lambda x: torch.tensor(np.ascontiguousarray(x), device=dev)  # noqa: E731
xyz = t(sc["means3D"])
feats = t(sc["colors"])
op = t(sc["opacities"])
scl = t(sc["scales"])
rot = t(sc["rotations"])
cp = {"image_height": torch.full((B,), W, device=dev), "image_width": torch.full((B,), W, device=dev),
      "tanfovx": t(np.array([c["tanfovx"] for c in cams], np.float32)),
      "tanfovy": t(np.array([c["tanfovy"] for c in cams], np.float32)),
      "view": t(np.stack([c["viewmatrix"] for c in cams])), "proj": t(np.stack([c["projmatrix"] for c in cams])),
      "campos": t(np.stack([c["campos"] for c in cams]))}
bg = torch.zeros((B, 32), device=dev)
mean2d = torch.zeros_like(xyz)


def run(n_rounds, record):
    ts, tc = 0.0, 0.0
    for _ in range(n_rounds):
        for bi in range(B):
            t0 = time.perf_counter()
            rs = GaussianRasterizationSettings(
                image_height=int(cp["image_height"][bi]), image_width=int(cp["image_width"][bi]),
                tanfovx=float(cp["tanfovx"][bi]), tanfovy=float(cp["tanfovy"][bi]), bg=bg[bi], scale_modifier=1.0,
                viewmatrix=cp["view"][bi], projmatrix=cp["proj"][bi], sh_degree=0, campos=cp["campos"][bi],
                prefiltered=False, debug=False, antialiasing=False)
            t1 = time.perf_counter()
            with torch.no_grad():
                GaussianRasterizer_32(raster_settings=rs)(means3D=xyz, means2D=mean2d, shs=None, colors_precomp=feats,
                                                          opacities=op, scales=scl, rotations=rot, cov3D_precomp=None)
            t2 = time.perf_counter()
            ts += t1 - t0
            tc += t2 - t1
    return ts, tc


run(2, False)
torch.cuda.synchronize()
n = 4
T0 = time.perf_counter()
ts, tc = run(n, True)
torch.cuda.synchronize()
T = time.perf_counter() - T0
frames = n * B
print(f"per frame: wall {1e6 * T / frames:.0f} us; settings incl. int()/float() syncs {1e6 * ts / frames:.0f} us; "
      f"rasterizer call (host) {1e6 * tc / frames:.0f} us")

if os.environ.get("FRAME_PROFILE"):
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    run(2, False)
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
