"""How far does the hardware-exp forward (split-bf16 products) land from the exact-exp one on the
contract workload? 32 config-2 frames through the batched entry, both modes; prints max |diff|,
the number of channel-pixels over 1e-4 and of n_contrib differences."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from guava_renderer_amd import _lib, scenes  # noqa: E402
from guava_renderer_amd.batch import BatchRasterizer  # noqa: E402

dev = torch.device("cuda:0")
B, P, W = 32, 100000, 512
sc = scenes.avatar_cloud(P, seed=0)
cams = scenes.frame_cameras(B, W, W, seed=1000)
t = lambda x: torch.tensor(np.ascontiguousarray(x), device=dev)  # noqa: E731
views = t(np.stack([c["viewmatrix"].reshape(16) for c in cams]))
projs = t(np.stack([c["projmatrix"].reshape(16) for c in cams]))
tanf = t(np.array([[c["tanfovx"], c["tanfovy"]] for c in cams], np.float32))
args = [t(sc[k]) for k in ("means3D", "colors", "opacities", "scales", "rotations")]
bgs = torch.zeros((B, 32), device=dev)
out = {}
for fast in (False, True):
    r = BatchRasterizer(B, P, W, W, R_capacity=24 * P * B, device=dev,
                        numerics=_lib.numerics(fast_exp=fast, split_bf16=True))
    col, inv, _ = r.forward(*args, views, projs, tanf, bgs)
    torch.cuda.synchronize()
    out[fast] = (col.clone(), inv.clone(), r.n_contrib().clone() if hasattr(r, "n_contrib") else None)
d = (out[True][0] - out[False][0]).abs()
print("max |dcol|", d.max().item(), "n > 1e-4:", int((d > 1e-4).sum()), "n > 1e-5:", int((d > 1e-5).sum()),
      "of", d.numel())
di = (out[True][1] - out[False][1]).abs()
print("max |dinvdepth|", di.max().item())
if out[True][2] is not None:
    print("n_contrib differences:", int((out[True][2] != out[False][2]).sum()))
