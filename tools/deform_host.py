"""Host (CPU) cost of the per-frame deform at B = 1 (AvatarPipeline.deform: EHMDeformer +
GaussianDeformer): issue time per call without synchronisation, and a cProfile of the Python side,
so the per-frame drop-in path's host-bound deform can be cut where it spends."""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
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
frames = [({k: v[i:i + 1] for k, v in w.bpt.items()}, {k: v[i:i + 1] for k, v in w.fpt.items()}) for i in range(w.B)]
N = 300


def run(fn, name):
    with torch.no_grad():
        for k in range(20):
            fn(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(N):
            fn(k)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    print(f"{name:24s} issue {1e6 * (t1 - t0) / N:7.1f} us/call   total {1e6 * (t2 - t0) / N:7.1f} us/call", flush=True)


run(lambda k: pipe.deform(*frames[k % len(frames)]), "deform (EHM + Gaussians)")
run(lambda k: pipe.ehm(*frames[k % len(frames)]), "EHM only")
e = pipe.ehm(*frames[0])
run(lambda k: pipe.gauss(e["vertices"], e["ver_transform_mat"]), "Gaussians only")

pr = cProfile.Profile()
with torch.no_grad():
    pr.enable()
    for k in range(N):
        pipe.deform(*frames[k % len(frames)])
    pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
