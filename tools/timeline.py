"""Dump the render_fwd work-item timeline of one C2 batch (instrumented kernel) to
gpurun_out/timeline.npz: per strip item (start, end [100 MHz ticks], k-steps, XCD)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from guava_renderer_amd import _lib, scenes  # noqa: E402
from guava_renderer_amd.batch import BatchRasterizer  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
P, W, H = 100000, 512, 512
dev = torch.device("cuda")
sc = scenes.avatar_cloud(P, seed=0)
cams = scenes.frame_cameras(B, W, H, seed=1000)
t = lambda x: torch.tensor(np.ascontiguousarray(x), device=dev)  # noqa: E731
args = (t(sc["means3D"]), t(sc["colors"]), t(sc["opacities"]), t(sc["scales"]), t(sc["rotations"]),
        t(np.stack([c["viewmatrix"].reshape(16) for c in cams])), t(np.stack([c["projmatrix"].reshape(16) for c in cams])),
        t(np.array([[c["tanfovx"], c["tanfovy"]] for c in cams], np.float32)), torch.zeros((B, 32), device=dev))
rast = BatchRasterizer(B, P, W, H, R_capacity=8 * P * B, device=dev)
rast.forward(*args)
torch.cuda.synchronize()
L = _lib.load()
cap = B * 1024 * 4
tl = torch.zeros((cap, 4), dtype=torch.int32, device=dev)
cnt = torch.zeros(8, dtype=torch.int64, device=dev)
L.gsr_render_timeline(tl.data_ptr(), cap)
rast.forward(*args)
torch.cuda.synchronize()
L.gsr_render_timeline(None, 0)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", os.environ.get("TL_OUT", "timeline.npz")), tl=tl.cpu().numpy(), cnt=cnt.cpu().numpy())
tl = tl.cpu().numpy()
tl = tl[tl[:, 1] != 0].astype(np.uint32).astype(np.int64)
tl[:, 1] += (tl[:, 1] < tl[:, 0]) * (1 << 32)  # 32-bit tick wrap inside an item
dur = tl[:, 1] - tl[:, 0]
span = tl[:, 1].max() - tl[:, 0].min()
print(f"items {len(tl)} span {span / 100:.1f} us, longest item {dur.max() / 100:.1f} us ({tl[dur.argmax(), 2]} k-steps), "
      f"mean {dur.mean() / 100:.1f} us, p99 {np.percentile(dur, 99) / 100:.1f} us, "
      f"items ending in the last 20% of the span: {int((tl[:, 1] > tl[:, 0].min() + 0.8 * span).sum())}")
order = np.argsort(-dur)[:8]
print("top items (start, dur us, ksteps):", [(round((tl[i, 0] - tl[:, 0].min()) / 100, 1), round(dur[i] / 100, 1), int(tl[i, 2])) for i in order])
