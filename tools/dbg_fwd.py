import sys, os, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
from helpers import make_scene, gpu_forward, oracle_forward
from guava_renderer_amd import _lib
_lib.set_exact_exp(True)
d = make_scene("random", 10000, 256, 256, seed=3)
g_col, g_radii, g_inv, gs = gpu_forward(d)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "dbg_fwd.npz"), col=g_col, nc=gs["n_contrib"], fT=gs["final_T"], pl=gs["point_list"], ext=gs["ext"])
print("saved")
