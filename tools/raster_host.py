"""Where the host time of GUAVA's per-frame drop-in render goes (gaussian_render.py:37-67 through
GaussianRasterizer_32): per frame, the time spent inside the C call gsr_forward_async (argument
checks, scratch fit and the kernel launches), in the rest of the Python call chain, and waiting in
the loop's device synchronisations (GUAVA's int()/float() camera reads).  The per-frame loop is
serial, so host time spent issuing launches is time the GPU waits."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from diff_gaussian_rasterization_32 import GaussianRasterizationSettings, GaussianRasterizer_32  # noqa: E402
from guava_renderer_amd import _lib  # noqa: E402
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
L = _lib.load()
inner = L.gsr_forward_async
acc = {"c": 0.0, "n": 0}


def timed(*a):
    t0 = time.perf_counter()
    r = inner(*a)
    acc["c"] += time.perf_counter() - t0
    acc["n"] += 1
    return r


L.gsr_forward_async = timed
N = 300


def loop(with_deform):
    dg0 = pipe.deform(*frames[0][:2])
    for k in range(N + 20):
        if k == 20:
            torch.cuda.synchronize()
            acc["c"], acc["n"] = 0.0, 0
            t0 = time.perf_counter()
        bp, fp, cam = frames[k % len(frames)]
        dg = pipe.deform(bp, fp) if with_deform else dg0
        a = {"xyz": dg["xyz"], "rotation": dg["rotation"], "scaling": dg["scaling"], "opacity": opacity,
             "features_color": colors}
        bench._render_model(a, cam, 1, dev, GaussianRasterizationSettings, GaussianRasterizer_32)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"{'deform + render' if with_deform else 'render only':16s} {1e6 * el / N:7.1f} us/frame; inside "
          f"gsr_forward_async {1e6 * acc['c'] / max(acc['n'], 1):6.1f} us/call ({acc['n']} calls)", flush=True)


with torch.no_grad():
    loop(False)
    loop(True)
    # the C call alone, back to back (no GUAVA glue, no syncs): its pure issue cost
    mean_3d = pipe.deform(*frames[0][:2])["xyz"][0]
    cam = frames[0][2]
    rs = GaussianRasterizationSettings(
        image_height=w.H, image_width=w.W, tanfovx=float(cam["tanfovx"][0]), tanfovy=float(cam["tanfovy"][0]),
        bg=torch.zeros(32, device=dev), scale_modifier=1.0, viewmatrix=cam["world_view_transform"][0],
        projmatrix=cam["full_proj_transform"][0], sh_degree=0, campos=cam["camera_center"][0], prefiltered=False,
        debug=False, antialiasing=False)
    r = GaussianRasterizer_32(raster_settings=rs)
    d0 = pipe.deform(*frames[0][:2])
    args = dict(means3D=mean_3d, means2D=torch.zeros_like(mean_3d), shs=None, colors_precomp=colors[0],
                opacities=opacity[0], scales=d0["scaling"][0], rotations=d0["rotation"][0], cov3D_precomp=None)
    for _ in range(20):
        r(**args)
    torch.cuda.synchronize()
    acc["c"], acc["n"] = 0.0, 0
    t0 = time.perf_counter()
    for _ in range(N):
        r(**args)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"rasterizer call alone: issue {1e6 * (t1 - t0) / N:6.1f} us/call (inside C {1e6 * acc['c'] / N:6.1f}), "
          f"GPU-bound total {1e6 * (t2 - t0) / N:6.1f} us/call", flush=True)

# cProfile of the rasterizer call alone (Python side; the C call counts as the caller's own time)
import cProfile  # noqa: E402
import pstats  # noqa: E402
with torch.no_grad():
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(N):
        r(**args)
    pr.disable()
    torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
