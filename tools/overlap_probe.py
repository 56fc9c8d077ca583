"""Probe: do two avatar batches in flight on two HIP streams (deform+binning of one overlapping the
render of the other) raise throughput over one stream?  Prints frames/s for 1 and 2 streams."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from guava_renderer_amd import avatar, scenes  # noqa: E402
from guava_renderer_amd.pipeline import AvatarPipeline  # noqa: E402

B, P, W, H = 32, 100000, 512, 512
dev = torch.device("cuda")
t = lambda x: torch.tensor(np.ascontiguousarray(x), device=dev)  # noqa: E731
body, flame, extra = avatar.ehm_assets(seed=0)
verts, faces, tex = avatar.template_mesh()
g = avatar.gaussians(verts, faces, tex, P=P, seed=0)
cams = scenes.frame_cameras(B, W, H, seed=1000)
views = t(np.stack([c["viewmatrix"].reshape(16) for c in cams]))
projs = t(np.stack([c["projmatrix"].reshape(16) for c in cams]))
tanf = t(np.array([[c["tanfovx"], c["tanfovy"]] for c in cams], np.float32))
bp, fp = avatar.ehm_params(B, seed=1000)
bpt = {k: t(v) for k, v in bp.items()}
fpt = {k: t(v) for k, v in fp.items()}
pipes = [AvatarPipeline(body, flame, extra, g, B, W, H, R_capacity=12 * P * B, device=dev) for _ in range(2)]
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
K = 20
for n in (1, 2):
    for i in range(4):
        with torch.cuda.stream(streams[i % n]):
            pipes[i % n].render(bpt, fpt, views, projs, tanf)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        with torch.cuda.stream(streams[i % n]):
            pipes[i % n].render(bpt, fpt, views, projs, tanf)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    assert not any(p.rast.status()[1] for p in pipes), "capacity overflow"
    print(f"streams={n}: {B * K / el:.0f} frames/s ({1000 * el / K:.3f} ms/step)", flush=True)
