"""Work-item timeline of the single-frame quad render (k_render_quad's TL variant through
gsr_render_timeline) on one C2 frame of GUAVA's drop-in path: the kernel's span, and for the longest
items their start / duration, 4-Gaussian steps, list refills and list entries walked -- what sets the
per-frame render time.  python tools/quad_timeline.py"""
import os
import sys

import numpy as np
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
bp = {k: v[1:2] for k, v in w.bpt.items()}
fp = {k: v[1:2] for k, v in w.fpt.items()}
cam = bench._cam_params(w, 1, lo=1)
dg = pipe.deform(bp, fp)
a = {"xyz": dg["xyz"], "rotation": dg["rotation"], "scaling": dg["scaling"],
     "opacity": pipe.gauss.opacity.unsqueeze(0), "features_color": pipe.gauss.colors.unsqueeze(0)}
L = _lib.load()
cap = 1 << 16
buf = torch.zeros((cap * 8,), dtype=torch.int32, device=dev)  # records, then the quad kernel's phase sums
with torch.no_grad():
    for _ in range(5):
        bench._render_model(a, cam, 1, dev, GaussianRasterizationSettings, GaussianRasterizer_32)
    torch.cuda.synchronize()
    L.gsr_render_timeline(buf.data_ptr(), cap | 0x80000000)  # (records + phase sums)
    bench._render_model(a, cam, 1, dev, GaussianRasterizationSettings, GaussianRasterizer_32)
    torch.cuda.synchronize()
    L.gsr_render_timeline(None, 0)
allr = buf.view(2 * cap, 4).cpu().numpy().astype(np.int64) & 0xFFFFFFFF
r, ph = allr[:cap], allr[cap:]
used = (r[:, 0] != 0) | (r[:, 1] != 0)
r = r[used]
ph = ph[used]
idx = np.nonzero(used)[0]
t0 = r[:, 0].min()
start, end = (r[:, 0] - t0) * 10.0, (r[:, 1] - t0) * 10.0  # ns (100 MHz ticks)
dur = end - start
steps, refills, walk = r[:, 2] & 0xFFFF, r[:, 2] >> 16, r[:, 3]
print(f"items {len(r)}; span {end.max() / 1000:.1f} us; mean duration {dur.mean() / 1000:.2f} us; "
      f"starts: p50 {np.percentile(start, 50) / 1000:.1f} us, p99 {np.percentile(start, 99) / 1000:.1f}, "
      f"max {start.max() / 1000:.1f}")
print("latest-ending items: item  start_us  dur_us  steps  refills  walked  ns/step  ns/refill")
for i in np.argsort(-end)[:15]:
    print(f"  {idx[i]:6d} {start[i] / 1000:8.1f} {dur[i] / 1000:7.1f} {steps[i]:6d} {refills[i]:7d} {walk[i]:7d} "
          f"{dur[i] / max(steps[i], 1):8.0f} {dur[i] / max(refills[i], 1):9.0f}")
print("longest items:")
for i in np.argsort(-dur)[:10]:
    print(f"  {idx[i]:6d} {start[i] / 1000:8.1f} {dur[i] / 1000:7.1f} {steps[i]:6d} {refills[i]:7d} {walk[i]:7d}")
print(f"sum of item durations {dur.sum() / 1000:.0f} us over {len(r)} items; "
      f"work-weighted: refills {refills.sum()}, steps {steps.sum()}")
A = np.stack([steps, refills, np.ones_like(steps)], 1).astype(np.float64)
coef = np.linalg.lstsq(A, dur, rcond=None)[0]
print(f"fit over items: duration = {coef[0]:.0f} ns/step + {coef[1]:.0f} ns/refill + {coef[2]:.0f} ns")
late = start > 60000
if late.any():
    coef2 = np.linalg.lstsq(A[late], dur[late], rcond=None)[0]
    print(f"items starting after 60 us ({late.sum()}): {coef2[0]:.0f} ns/step + {coef2[1]:.0f} ns/refill + {coef2[2]:.0f}")
ph_steps = np.maximum(steps, 1)[:, None]
lt = np.argsort(-end)[:20]
print("latest-ending 20 items, core cycles per step: issue+refill %.0f, next alpha (records' wait) %.0f, "
      "blend+MFMA %.0f" % tuple((ph[lt, :3] / ph_steps[lt]).mean(0)))
print("all items: %.0f / %.0f / %.0f cycles per step" % tuple(ph[:, :3].sum(0) / max(steps.sum(), 1)))
