"""Where GUAVA's per-frame drop-in path (bench.py per_frame_dropin: deform at B=1 + one
GaussianRasterizer_32 call per frame) spends its time: wall time per frame of the whole loop, of the
deform alone, of the rasterizer call alone, and the GPU time of each (HIP events), N frames each."""
import os
import sys
import time

import numpy as np
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
N = 200


def timeit(name, fn):
    with torch.no_grad():
        for k in range(10):
            fn(k)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for k in range(N):
            fn(k)
        e1.record()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    print(f"{name:28s} wall {1e3 * el / N:7.3f} ms/frame   (events {e0.elapsed_time(e1) / N:7.3f})", flush=True)


assets0 = None


def deform(k):
    bp, fp, _ = frames[k % len(frames)]
    return pipe.deform(bp, fp)


dg = deform(0)
assets0 = {"xyz": dg["xyz"].clone(), "rotation": dg["rotation"].clone(), "scaling": dg["scaling"].clone(),
           "opacity": pipe.gauss.opacity.unsqueeze(0), "features_color": pipe.gauss.colors.unsqueeze(0)}


def render(k):
    return bench._render_model(assets0, frames[k % len(frames)][2], 1, dev, GaussianRasterizationSettings,
                               GaussianRasterizer_32)


def full(k):
    bp, fp, cam = frames[k % len(frames)]
    d = pipe.deform(bp, fp)
    a = {"xyz": d["xyz"], "rotation": d["rotation"], "scaling": d["scaling"], "opacity": assets0["opacity"],
         "features_color": assets0["features_color"]}
    return bench._render_model(a, cam, 1, dev, GaussianRasterizationSettings, GaussianRasterizer_32)


timeit("deform (B=1)", deform)
timeit("render (drop-in, B=1)", render)
timeit("deform + render", full)
if len(sys.argv) > 1 and sys.argv[1] == "stages":
    from guava_renderer_amd.batch import profile_enable, profile_read
    profile_enable(("preprocess", "scan", "depth_sort", "chunk_count", "tile_scan", "ordered_scatter", "render_fwd"))
    with torch.no_grad():
        for k in range(N):
            render(k)
    torch.cuda.synchronize()
    print({k: round(v[0] / max(v[1], 1), 4) for k, v in profile_read().items()})
