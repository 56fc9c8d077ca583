"""Where the GPU Gaussian assembly departs from the float64 oracle (rotation error vs index class,
decision margin and face conditioning):  python tools/diag_deform.py [P] [gpt] [B] [cross]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import lbs_oracle as lo  # noqa: E402
from guava_renderer_amd import avatar  # noqa: E402
from guava_renderer_amd.pipeline import AvatarPipeline  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 300000
gpt = int(sys.argv[2]) if len(sys.argv) > 2 else 3
B = int(sys.argv[3]) if len(sys.argv) > 3 else 2
cross = len(sys.argv) > 4 and sys.argv[4] == "1"
body, flame, extra = avatar.ehm_assets(seed=0)
verts, faces, tex = avatar.template_mesh()
g = avatar.gaussians(verts, faces, tex * gpt, P=P, seed=0)
bp, fp = avatar.ehm_params(B, seed=2000)
if cross:
    sb, sf = avatar.ehm_params(1, seed=77)
    bp, fp = avatar.change_id_info(bp, fp, sb, sf)
dev = torch.device("cuda:0")
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
pipe = AvatarPipeline(body, flame, extra, g, B, 512, 512, R_capacity=1024, device=dev)
d = pipe.deform({k: t(v) for k, v in bp.items()}, {k: t(v) for k, v in fp.items()})
e = lo.ehm_forward(body, flame, extra, bp, fp)
ge = pipe.ehm({k: t(v) for k, v in bp.items()}, {k: t(v) for k, v in fp.items()})
print("verts max err", np.abs(ge["vertices"].cpu().numpy() - e["vertices"]).max(),
      "T max err", np.abs(ge["ver_transform_mat"].cpu().numpy() - e["ver_transform_mat"]).max())
ref = lo.deform_gaussians(e["vertices"], e["ver_transform_mat"], extra["faces"], g["vtx_rotations"],
                          g["vtx_scales"], g["binding_face"], g["face_bary"], g["local_xyz"],
                          g["uv_rotations"], g["uv_scales"])
q, rq = d["rotation"].cpu().numpy(), ref["rotation"]
err = np.minimum(np.abs(q - rq).max(-1), np.abs(q + rq).max(-1))
V = verts.shape[0]
print("xyz err", np.abs(d["xyz"].cpu().numpy() - ref["xyz"]).max())
print("rot err vertex", err[:, :V].max(), "uv", err[:, V:].max())
for thr in (1e-5, 2e-5, 1e-4, 1e-3):
    print(f"  > {thr}: vertex {(err[:, :V] > thr).sum()} uv {(err[:, V:] > thr).sum()}")
bad = np.argwhere(err > 2e-5)[:10]
for b_, i in bad:
    f = g["binding_face"][i - V] if i >= V else -1
    print(f"  frame {b_} gaussian {i} ({'uv' if i >= V else 'vtx'}) face {f} err {err[b_, i]:.3g} margin {ref['margin'][b_, i]:.3g}"
          f" q {q[b_, i]} ref {rq[b_, i]}")
