"""Times render_fwd variants (ablation switches) in one process: python tools/ablate.py"""
import sys, os, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from guava_renderer_amd import _lib, scenes
from guava_renderer_amd.batch import BatchRasterizer, profile_enable, profile_read
L = _lib.load()
B, P, W, H = 32, 100000, 512, 512
sc = scenes.avatar_cloud(P, seed=0)
cams = scenes.frame_cameras(B, W, H, seed=1000)
dev = torch.device("cuda")
t = lambda x: torch.tensor(np.ascontiguousarray(x), device=dev)
args = [t(sc["means3D"]), t(sc["colors"]), t(sc["opacities"]), t(sc["scales"]), t(sc["rotations"]),
        t(np.stack([c["viewmatrix"].reshape(16) for c in cams])), t(np.stack([c["projmatrix"].reshape(16) for c in cams])),
        t(np.array([[c["tanfovx"], c["tanfovy"]] for c in cams], np.float32)), torch.zeros((B, 32), device=dev)]
r = BatchRasterizer(B, P, W, H, R_capacity=30 * P * B)
variants = [(0, 1), (0, 0), (1, 1), (2, 1), (4, 1), (3, 1), (7, 1)]
res = {v: [] for v in variants}
for rep in range(3):
    for flags, exact in variants:
        L.gsr_debug_flags(flags); _lib.set_exact_exp(bool(exact))
        r.forward(*args); torch.cuda.synchronize()
        profile_read(); profile_enable(("render_fwd", "tile_sort"))
        for _ in range(3): r.forward(*args)
        torch.cuda.synchronize()
        p = profile_read(); profile_enable(())
        res[(flags, exact)].append(p["render_fwd"][0] / p["render_fwd"][1])
L.gsr_debug_flags(0); _lib.set_exact_exp(True)
names = {1: "noMFMA", 2: "noStageLoads", 4: "noBlend(cull only)"}
for (flags, exact), v in res.items():
    nm = "+".join(n for b, n in names.items() if flags & b) or "full"
    print(f"{nm:28s} exact={exact}  render_fwd ms/32 frames: min {min(v):.3f} med {np.median(v):.3f}")
