"""Host-side cost of GUAVA's per-frame caller (bench.py _render_model at B=1 + the deform), split
into its Python phases, each timed with the GPU idle before it (synchronised), N frames:
  cam reads    -- GaussianRasterizationSettings with int()/float() of four device scalars
  raster call  -- GaussianRasterizer_32(...)(...) until it returns (launches queued, no wait)
  deform call  -- AvatarPipeline.deform (B=1) until it returns
  gpu raster   -- the raster call's GPU time after it returns (synchronise)
python tools/frame_host.py"""
import os
import sys
import time

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
N = int(os.environ.get("N", "200"))
acc = {k: 0.0 for k in ("deform call", "deform gpu", "cam reads", "prep", "raster call", "gpu raster", "stack")}
with torch.no_grad():
    for k in range(N + 10):
        bp, fp, cam = frames[k % len(frames)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dg = pipe.deform(bp, fp)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        mean_3d = dg["xyz"]
        features_color = colors.clone()
        mean_2d = torch.zeros_like(mean_3d, dtype=torch.float32, requires_grad=True, device=dev)
        bg = torch.ones((1, features_color.shape[-1]), dtype=torch.float32, device=dev) * 0.0
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        rs = GaussianRasterizationSettings(
            image_height=int(cam["image_height"][0]), image_width=int(cam["image_width"][0]),
            tanfovx=float(cam["tanfovx"][0]), tanfovy=float(cam["tanfovy"][0]), bg=bg[0], scale_modifier=1.0,
            viewmatrix=cam["world_view_transform"][0], projmatrix=cam["full_proj_transform"][0], sh_degree=0,
            campos=cam["camera_center"][0], prefiltered=False, debug=False, antialiasing=False)
        t4 = time.perf_counter()
        img, rad, dep = GaussianRasterizer_32(raster_settings=rs)(
            means3D=mean_3d[0], means2D=mean_2d[0], shs=None, colors_precomp=features_color[0],
            opacities=opacity[0], scales=dg["scaling"][0], rotations=dg["rotation"][0], cov3D_precomp=None)
        t5 = time.perf_counter()
        torch.cuda.synchronize()
        t6 = time.perf_counter()
        out = torch.stack([img], 0), torch.stack([rad], 0), torch.stack([dep], 0)
        torch.cuda.synchronize()
        t7 = time.perf_counter()
        if k >= 10:
            for key, v in (("deform call", t1 - t0), ("deform gpu", t2 - t1), ("prep", t3 - t2), ("cam reads", t4 - t3),
                           ("raster call", t5 - t4), ("gpu raster", t6 - t5), ("stack", t7 - t6)):
                acc[key] += v
print({k: round(1e6 * v / N, 1) for k, v in acc.items()}, "us per frame (each phase after a synchronise)")
