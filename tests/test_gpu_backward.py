"""GPU parity of the backward path (render backward + projection backward) against the CPU oracle.

Gradients are summed in a different order on the GPU (wave reductions + float atomics) and the
32-channel "colour behind" recurrence is carried as a dot product, so the bar is a tolerance:
for every gradient tensor, max|gpu - oracle| <= 1e-4 * max|oracle| (plus an elementwise check).
The forward state the backward consumes (radii, tile lists, n_contrib, final_T) is bit-exact.
"""
import numpy as np
import pytest
import torch

from helpers import make_scene, oracle_forward, torch_inputs

pytestmark = pytest.mark.gpu

NAMES = ("means2D", "colors", "opacity", "means3D", "cov3D", "sh", "scales", "rotations")


def _gpu_backward(d, dL, dLinv, antialiasing=False, use_cov=None, numerics=0):
    from guava_renderer_amd.diff_gaussian_rasterization_32 import _C
    t = torch_inputs(d)
    empty = torch.Tensor([])
    cov = empty if use_cov is None else torch.tensor(use_cov, device="cuda")
    scales = t["scales"] if use_cov is None else empty
    rots = t["rotations"] if use_cov is None else empty
    R, color, radii, gb, bb, ib, invd = _C.rasterize_gaussians(
        t["bg"], t["means3D"], t["colors"], t["opacities"], scales, rots, 1.0, cov,
        t["viewmatrix"], t["projmatrix"], d["tanfovx"], d["tanfovy"], d["image_height"],
        d["image_width"], empty, 0, t["campos"], False, antialiasing, False, numerics=numerics)
    dLt = torch.tensor(dL, device="cuda")
    dLi = torch.tensor(dLinv, device="cuda") if dLinv is not None else torch.zeros((0, 1), device="cuda")
    grads = _C.rasterize_gaussians_backward(
        t["bg"], t["means3D"], radii, t["colors"], t["opacities"], scales, rots, 1.0, cov,
        t["viewmatrix"], t["projmatrix"], d["tanfovx"], d["tanfovy"], dLt, dLi, empty, 0, t["campos"],
        gb, R, bb, ib, antialiasing, False, numerics=numerics)
    torch.cuda.synchronize()
    return [g.cpu().numpy() for g in grads]


def _oracle_backward(d, dL, dLinv, antialiasing=False, use_cov=None):
    import oracle
    _, _, _, st = oracle.forward(
        d["means3D"], d["colors"], d["opacities"], None if use_cov is not None else d["scales"],
        None if use_cov is not None else d["rotations"], use_cov, d["viewmatrix"], d["projmatrix"],
        d["image_width"], d["image_height"], d["tanfovx"], d["tanfovy"], d["bg"],
        antialiasing=antialiasing)
    return oracle.backward(st, d["means3D"], d["colors"], d["opacities"],
                           None if use_cov is not None else d["scales"],
                           None if use_cov is not None else d["rotations"], use_cov,
                           d["viewmatrix"], d["projmatrix"], d["image_width"], d["image_height"],
                           d["tanfovx"], d["tanfovy"], d["bg"], dL, dLinv,
                           antialiasing=antialiasing)


def _check(g, o, tol=1e-4, skip=()):
    for name, a, b in zip(NAMES, g, o):
        if name in skip or b.size == 0:
            continue
        a = a.reshape(b.shape)
        scale = max(np.abs(b).max(), 1e-20)
        err = np.abs(a - b).max() / scale
        assert err <= tol, f"{name}: max err {err:.3g} (scale {scale:.3g})"


@pytest.mark.parametrize("kind,P,W,H,seed", [("random", 2000, 96, 64, 1), ("random", 6000, 160, 128, 2),
                                             ("avatar", 12000, 128, 128, 3)])
def test_backward_matches_oracle(kind, P, W, H, seed):
    d = make_scene(kind, P, W, H, seed=seed)
    rng = np.random.default_rng(seed)
    dL = rng.normal(size=(32, H, W)).astype(np.float32)
    dLinv = rng.normal(size=(1, H, W)).astype(np.float32)
    _check(_gpu_backward(d, dL, dLinv), _oracle_backward(d, dL, dLinv))


@pytest.mark.parametrize("kind,P,W,H,seed", [("random", 2000, 96, 64, 1), ("avatar", 12000, 128, 128, 3)])
def test_backward_split_bf16_matches_oracle(kind, P, W, H, seed):
    """GSR_NUMERICS_SPLIT_BF16: the backward's g = f . dL/dpixel contraction on split-bf16 MFMAs (the
    single-frame feature table pre-split by k_split_features) -- same 1e-4 bar."""
    from guava_renderer_amd import _lib
    d = make_scene(kind, P, W, H, seed=seed)
    rng = np.random.default_rng(seed)
    dL = rng.normal(size=(32, H, W)).astype(np.float32)
    dLinv = rng.normal(size=(1, H, W)).astype(np.float32)
    g = _gpu_backward(d, dL, dLinv, numerics=_lib.numerics(split_bf16=True))
    _check(g, _oracle_backward(d, dL, dLinv))


def test_backward_no_invdepth_grad():
    d = make_scene("random", 3000, 96, 96, seed=4)
    rng = np.random.default_rng(4)
    dL = rng.normal(size=(32, 96, 96)).astype(np.float32)
    _check(_gpu_backward(d, dL, None), _oracle_backward(d, dL, None))


def test_backward_antialiasing():
    d = make_scene("random", 3000, 96, 80, seed=5)
    rng = np.random.default_rng(5)
    dL = rng.normal(size=(32, 80, 96)).astype(np.float32)
    dLinv = rng.normal(size=(1, 80, 96)).astype(np.float32)
    _check(_gpu_backward(d, dL, dLinv, antialiasing=True), _oracle_backward(d, dL, dLinv, antialiasing=True))


def test_backward_precomputed_cov3D():
    import oracle
    d = make_scene("random", 2000, 80, 80, seed=6)
    st = oracle.preprocess(d["means3D"], d["scales"], d["rotations"], d["opacities"], None,
                           d["viewmatrix"], d["projmatrix"], 80, 80, d["tanfovx"], d["tanfovy"])
    cov = st["cov3D"].copy()
    rng = np.random.default_rng(6)
    dL = rng.normal(size=(32, 80, 80)).astype(np.float32)
    dLinv = np.zeros((1, 80, 80), np.float32)
    g = _gpu_backward(d, dL, dLinv, use_cov=cov)
    o = _oracle_backward(d, dL, dLinv, use_cov=cov)
    _check(g, o, skip=("scales", "rotations"))
    assert np.all(g[6] == 0) and np.all(g[7] == 0)


def test_autograd_through_drop_in_api():
    """Gradients flow through GaussianRasterizer_32 exactly as through the reference autograd
    Function: every input gets the _C backward's tensor, means2D gets the screen-space grad."""
    from diff_gaussian_rasterization_32 import GaussianRasterizationSettings, GaussianRasterizer_32
    d = make_scene("avatar", 8000, 96, 96, seed=7)
    t = torch_inputs(d, requires_grad=True)
    means2D = torch.zeros_like(t["means3D"], requires_grad=True)
    s = GaussianRasterizationSettings(96, 96, d["tanfovx"], d["tanfovy"], t["bg"], 1.0,
                                      t["viewmatrix"], t["projmatrix"], 0, t["campos"], False,
                                      False, False)
    color, radii, invd = GaussianRasterizer_32(s)(
        means3D=t["means3D"], means2D=means2D, opacities=t["opacities"], colors_precomp=t["colors"],
        scales=t["scales"], rotations=t["rotations"])
    rng = np.random.default_rng(7)
    dL = rng.normal(size=(32, 96, 96)).astype(np.float32)
    (color * torch.tensor(dL, device="cuda")).sum().backward()
    o = _oracle_backward(d, dL, np.zeros((1, 96, 96), np.float32))
    g = [means2D.grad, t["colors"].grad, t["opacities"].grad, t["means3D"].grad, None, None,
         t["scales"].grad, t["rotations"].grad]
    for name, a, b in zip(NAMES, g, o):
        if a is None:
            continue
        a = a.cpu().numpy().reshape(b.shape)
        err = np.abs(a - b).max() / max(np.abs(b).max(), 1e-20)
        assert err <= 1e-4, (name, err)
