"""Golden fixtures (tests/golden/oracle_micro.npz, written by tests/golden/make_golden.py).

CPU: the oracle reproduces the committed forward state, image and gradients bit-exactly.
GPU: the HIP path reproduces the committed forward outputs bit-exactly (exact-exp mode) and the
gradients within 1e-4 of their scale.
"""
import os

import numpy as np
import pytest

import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = np.load(os.path.join(HERE, "golden", "oracle_micro.npz"))
SCENES = sorted({k.split("__")[0] for k in GOLD.files})


def _scene(name):
    g = {k.split("__", 1)[1]: GOLD[k] for k in GOLD.files if k.startswith(name + "__")}
    W, H = (int(v) for v in g["in_size"])
    d = dict(means3D=g["in_means3D"], colors=g["in_colors"], opacities=g["in_opacities"],
             scales=g["in_scales"], rotations=g["in_rotations"], viewmatrix=g["in_viewmatrix"],
             projmatrix=g["in_projmatrix"], campos=g["in_campos"], bg=g["in_bg"],
             tanfovx=float(g["in_tan"][0]), tanfovy=float(g["in_tan"][1]), image_width=W, image_height=H)
    return d, g


@pytest.mark.parametrize("name", SCENES)
def test_oracle_reproduces_golden(name):
    d, g = _scene(name)
    W, H = d["image_width"], d["image_height"]
    col, radii, invd, st = oracle.forward(d["means3D"], d["colors"], d["opacities"], d["scales"],
                                          d["rotations"], None, d["viewmatrix"], d["projmatrix"], W, H,
                                          d["tanfovx"], d["tanfovy"], d["bg"])
    np.testing.assert_array_equal(col, g["out_color"])
    np.testing.assert_array_equal(invd, g["out_invdepth"])
    np.testing.assert_array_equal(radii, g["out_radii"])
    for k in ("means2D", "depths", "conic_opacity", "tiles_touched", "point_list", "ranges", "final_T",
              "n_contrib"):
        np.testing.assert_array_equal(st[k], g["st_" + k], err_msg=k)
    grads = oracle.backward(st, d["means3D"], d["colors"], d["opacities"], d["scales"], d["rotations"], None,
                            d["viewmatrix"], d["projmatrix"], W, H, d["tanfovx"], d["tanfovy"], d["bg"],
                            g["in_dL"], g["in_dLinv"])
    for nm, v in zip(("means2D", "colors", "opacity", "means3D", "cov3D", "sh", "scales", "rotations"), grads):
        np.testing.assert_array_equal(v, g["grad_" + nm], err_msg=nm)


@pytest.mark.gpu
@pytest.mark.parametrize("name", SCENES)
def test_gpu_matches_golden(name):
    import torch
    from helpers import gpu_forward, torch_inputs
    from guava_renderer_amd.diff_gaussian_rasterization_32 import _C
    d, g = _scene(name)
    W, H = d["image_width"], d["image_height"]
    col, radii, invd, st = gpu_forward(d)
    np.testing.assert_array_equal(col, g["out_color"])
    np.testing.assert_array_equal(invd, g["out_invdepth"])
    np.testing.assert_array_equal(radii, g["out_radii"])
    np.testing.assert_array_equal(st["n_contrib"], g["st_n_contrib"])
    np.testing.assert_array_equal(st["point_list"][:st["R"]], g["st_point_list"])
    # backward through the native surface
    t = torch_inputs(d)
    empty = torch.Tensor([])
    R, color, rad, gb, bb, ib, _ = _C.rasterize_gaussians(
        t["bg"], t["means3D"], t["colors"], t["opacities"], t["scales"], t["rotations"], 1.0, empty,
        t["viewmatrix"], t["projmatrix"], d["tanfovx"], d["tanfovy"], H, W, empty, 0, t["campos"], False,
        False, False)
    grads = _C.rasterize_gaussians_backward(
        t["bg"], t["means3D"], rad, t["colors"], t["opacities"], t["scales"], t["rotations"], 1.0, empty,
        t["viewmatrix"], t["projmatrix"], d["tanfovx"], d["tanfovy"], torch.tensor(g["in_dL"], device="cuda"),
        torch.tensor(g["in_dLinv"], device="cuda"), empty, 0, t["campos"], gb, R, bb, ib, False, False)
    for nm, v in zip(("means2D", "colors", "opacity", "means3D", "cov3D", "sh", "scales", "rotations"), grads):
        ref = g["grad_" + nm]
        if ref.size == 0:
            continue
        a = v.cpu().numpy().reshape(ref.shape)
        err = np.abs(a - ref).max() / max(np.abs(ref).max(), 1e-20)
        assert err <= 1e-4, (nm, err)
