"""cProfile of the per-frame drop-in loop's host side (deform B=1 + GaussianRasterizer_32), N frames:
prints the functions with the most own time.  python tools/frame_cprofile.py"""
import cProfile
import os
import pstats
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from diff_gaussian_rasterization_32 import GaussianRasterizationSettings, GaussianRasterizer_32  # noqa: E402
from guava_renderer_amd.pipeline import AvatarPipeline  # noqa: E402

dev = torch.device("cuda:0")


class A:
    pipeline = "avatar"
    config = "c2"
    inflight = 1
    refine = False


w = bench.Workload(A, bench._workload("c2"), 8, 0, 8, dev, 0)
body, flame, extra, g = w.avatar_assets
pipe = AvatarPipeline(body, flame, extra, g, 1, w.W, w.H, R_capacity=1024, device=dev)
frames = [({k: v[i:i + 1] for k, v in w.bpt.items()}, {k: v[i:i + 1] for k, v in w.fpt.items()},
           bench._cam_params(w, 1, lo=i)) for i in range(w.B)]
opacity, colors = pipe.gauss.opacity.unsqueeze(0), pipe.gauss.colors.unsqueeze(0)


def frame(k):
    bp, fp, cam = frames[k % len(frames)]
    d = pipe.deform(bp, fp)
    a = {"xyz": d["xyz"], "rotation": d["rotation"], "scaling": d["scaling"], "opacity": opacity,
         "features_color": colors}
    return bench._render_model(a, cam, 1, dev, GaussianRasterizationSettings, GaussianRasterizer_32)


N = int(os.environ.get("N", "300"))
with torch.no_grad():
    for k in range(20):
        frame(k)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for k in range(N):
        frame(k)
    torch.cuda.synchronize()
    pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(28)
