import sys, os, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from guava_renderer_amd import _lib, scenes
from guava_renderer_amd.batch import BatchRasterizer
L = _lib.load()
_lib.set_exact_exp(True)
B, P, W, H = 32, 100000, 512, 512
sc = scenes.avatar_cloud(P, seed=0)
cams = scenes.frame_cameras(B, W, H, seed=1000)
dev = torch.device("cuda")
t = lambda x: torch.tensor(np.ascontiguousarray(x), device=dev)
args = [t(sc["means3D"]), t(sc["colors"]), t(sc["opacities"]), t(sc["scales"]), t(sc["rotations"]),
        t(np.stack([c["viewmatrix"].reshape(16) for c in cams])), t(np.stack([c["projmatrix"].reshape(16) for c in cams])),
        t(np.array([[c["tanfovx"], c["tanfovy"]] for c in cams], np.float32)), torch.zeros((B, 32), device=dev)]
r = BatchRasterizer(B, P, W, H, R_capacity=30 * P * B)
r.forward(*args)
T = (W // 16) * (H // 16)
stats = torch.zeros((B * T * 4, 8), dtype=torch.int32, device=dev)
L.gsr_debug_render_stats(stats.data_ptr())
r.forward(*args); torch.cuda.synchronize()
L.gsr_debug_render_stats(None)
s = stats.cpu().numpy().astype(np.int64)
np.save(os.path.join(ROOT, "gpurun_out", "render_stats.npy"), s)
cyc, rounds, surv, n = s[:, 0], s[:, 1], s[:, 2], s[:, 3]
busy = n > 0
print("tiles*waves busy", busy.sum(), "of", len(n))
print("cycles: mean %.0f p50 %.0f p99 %.0f max %.0f" % (cyc[busy].mean(), np.median(cyc[busy]), np.percentile(cyc[busy], 99), cyc.max()))
print("rounds: mean %.1f max %d ; surv per wave mean %.1f total %d" % (rounds[busy].mean(), rounds.max(), surv[busy].mean(), surv.sum()))
print("cycles per round %.0f ; cycles per surviving G %.1f" % (cyc[busy].sum() / max(rounds[busy].sum(), 1), cyc[busy].sum() / max(surv.sum(), 1)))
print("sum cycles (wave-lifetimes) %.3g" % cyc.sum())

rs, re_ = s[:, 4], s[:, 5]
t0 = rs.min()
rs = rs - t0; re_ = re_ - t0
print("realtime span (us) %.1f" % (re_.max() / 100.0))
# concurrency profile of busy waves over time (100 MHz ticks)
grid = np.arange(0, re_.max(), max(1, re_.max() // 50))
conc = [((rs <= g) & (re_ > g) & busy).sum() for g in grid]
print("busy waves resident over time:", conc)
concall = [((rs <= g) & (re_ > g)).sum() for g in grid]
print("all waves resident over time:", concall)
hw = s[:, 6]; xcc = s[:, 7]
cu = (hw >> 8) & 0xF; sh = (hw >> 12) & 1; se = (hw >> 13) & 0x7
print("xcc ids", np.unique(xcc & 0xF), "se", np.unique(se), "cu", np.unique(cu))
