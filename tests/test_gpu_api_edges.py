"""Edge cases of the drop-in API on the GPU.

* markVisible (rasterize_points.cu:225-244, rasterizer_impl.cu:54-66,141-153): `_C.mark_visible` and
  `GaussianRasterizer_32.markVisible` bit-exact with the oracle (view-space z > 0.2), including
  points behind the camera and on the near plane.
* A frame where every Gaussian is culled (P > 0, R = 0): the output is exactly the background
  (the drop-in path allocates out_color with torch.empty, so every pixel must be written), radii
  and inverse depth 0 -- through `_C` and through the batched entry.
* Batched inputs with stride-0 frames (deform.py's expanded features_color / opacity) or
  non-contiguous rows render exactly like contiguous copies.
* The refiner head's prepared-feature cache follows tensor identity, not the address.
"""
import numpy as np
import pytest
import torch

from helpers import make_scene, torch_inputs

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _world_z_for_view_z(d, m, zv):
    """World z that puts points (x, y from m) at view-space depth zv (row-vector view matrix,
    graphics_utils.py:44-50 layout: z_view = x V[0][2] + y V[1][2] + z V[2][2] + V[3][2])."""
    V = d["viewmatrix"].astype(np.float64).reshape(4, 4)
    z = (zv - m[:, 0] * V[0, 2] - m[:, 1] * V[1, 2] - V[3, 2]) / V[2, 2]
    return z.astype(np.float32)


def test_mark_visible_bit_exact():
    import oracle
    from diff_gaussian_rasterization_32 import GaussianRasterizationSettings, GaussianRasterizer_32
    from guava_renderer_amd.diff_gaussian_rasterization_32 import _C
    d = make_scene("random", 5000, 64, 64, seed=21)
    m = d["means3D"].copy()
    # put some points behind the camera and around the near plane (view-space z in [-1, 1], and 0.2)
    m[:500, 2] = _world_z_for_view_z(d, m[:500], np.linspace(-1.0, 1.0, 500))
    m[500:520, 2] = _world_z_for_view_z(d, m[500:520], np.full(20, 0.2))
    t = torch_inputs(d)
    mt = torch.tensor(m, device=DEV)
    got = _C.mark_visible(mt, t["viewmatrix"], t["projmatrix"]).cpu().numpy()
    ref = oracle.mark_visible(m, d["viewmatrix"], d["projmatrix"])
    np.testing.assert_array_equal(got, ref)
    assert 0 < ref.sum() < len(ref)
    s = GaussianRasterizationSettings(64, 64, d["tanfovx"], d["tanfovy"], t["bg"], 1.0, t["viewmatrix"],
                                      t["projmatrix"], 0, t["campos"], False, False, False)
    vis = GaussianRasterizer_32(s).markVisible(mt)
    assert vis.dtype == torch.bool
    np.testing.assert_array_equal(vis.cpu().numpy(), ref)


def test_all_culled_frame_is_background():
    from guava_renderer_amd.batch import BatchRasterizer
    from guava_renderer_amd.diff_gaussian_rasterization_32 import _C
    d = make_scene("random", 3000, 80, 48, seed=22)
    d["means3D"][:, 2] = _world_z_for_view_z(d, d["means3D"], np.full(3000, -3.0))  # all behind the camera
    bg = np.linspace(-1.0, 2.0, 32).astype(np.float32)
    t = torch_inputs(d)
    t["bg"] = torch.tensor(bg, device=DEV)
    empty = torch.Tensor([])
    R, color, radii, gb, bb, ib, invd = _C.rasterize_gaussians(
        t["bg"], t["means3D"], t["colors"], t["opacities"], t["scales"], t["rotations"], 1.0, empty,
        t["viewmatrix"], t["projmatrix"], d["tanfovx"], d["tanfovy"], 48, 80, empty, 0, t["campos"],
        False, False, False)
    torch.cuda.synchronize()
    assert R == 0
    expect = np.broadcast_to(bg[:, None, None], (32, 48, 80))
    np.testing.assert_array_equal(color.cpu().numpy(), expect)
    assert (radii.cpu().numpy() == 0).all() and (invd.cpu().numpy() == 0).all()
    # batched entry, 2 frames
    r = BatchRasterizer(2, 3000, 80, 48, R_capacity=1024, device=DEV)
    view = t["viewmatrix"].reshape(1, 16).expand(2, 16).contiguous()
    proj = t["projmatrix"].reshape(1, 16).expand(2, 16).contiguous()
    tanf = torch.tensor([[d["tanfovx"], d["tanfovy"]]] * 2, device=DEV)
    col, inv, rad = r.forward(t["means3D"], t["colors"], t["opacities"], t["scales"], t["rotations"], view,
                              proj, tanf, t["bg"])
    r.poll(wait=True)
    np.testing.assert_array_equal(col.cpu().numpy(), np.broadcast_to(expect, (2, 32, 48, 80)))
    assert (rad.cpu().numpy() == 0).all() and (inv.cpu().numpy() == 0).all()


def _cams(n, W, H):
    from guava_renderer_amd import scenes
    cams = scenes.frame_cameras(n, W, H, seed=1000)
    t = lambda x: torch.tensor(np.ascontiguousarray(x), device=DEV)  # noqa: E731
    return (t(np.stack([c["viewmatrix"].reshape(16) for c in cams])),
            t(np.stack([c["projmatrix"].reshape(16) for c in cams])),
            t(np.array([[c["tanfovx"], c["tanfovy"]] for c in cams], np.float32)))


def test_batched_inputs_follow_tensor_strides():
    from guava_renderer_amd import scenes
    from guava_renderer_amd.batch import BatchRasterizer
    B, P, W = 3, 20000, 128
    sc = scenes.avatar_cloud(P, seed=4)
    views, projs, tanf = _cams(B, W, W)
    t = lambda x: torch.tensor(np.ascontiguousarray(x), device=DEV)  # noqa: E731
    means = t(sc["means3D"])
    cols, opac = t(sc["colors"]), t(sc["opacities"])
    scales, rots = t(sc["scales"]), t(sc["rotations"])
    bg = torch.zeros((B, 32), device=DEV)
    ref = BatchRasterizer(B, P, W, W, R_capacity=16 * P * B, device=DEV)
    c_ref, i_ref, r_ref = [x.clone() for x in ref.forward(means, cols, opac, scales, rots, views, projs, tanf, bg)]
    r = BatchRasterizer(B, P, W, W, R_capacity=16 * P * B, device=DEV)
    # deform.py's layout: per-frame geometry [B,P,k], features / opacity expanded (frame stride 0)
    m3 = means.unsqueeze(0).repeat(B, 1, 1)
    c_exp = cols.unsqueeze(0).expand(B, -1, -1)
    o_exp = opac.unsqueeze(0).expand(B, -1, -1)
    # rotations as a non-contiguous view ([B,P,4] slice of a wider buffer)
    wide = torch.zeros((B, P, 6), device=DEV)
    wide[..., 1:5] = rots
    r_view = wide[..., 1:5]
    s3 = scales.unsqueeze(0).repeat(B, 1, 1)
    c1, i1, r1 = r.forward(m3, c_exp, o_exp, s3, r_view, views, projs, tanf, bg[:1].expand(B, -1))
    torch.cuda.synchronize()
    assert torch.equal(c1, c_ref) and torch.equal(i1, i_ref) and torch.equal(r1, r_ref)
    with pytest.raises(ValueError):
        r.forward(means[:10], cols, opac, scales, rots, views, projs, tanf, bg)
    with pytest.raises(TypeError):
        r.forward(means.double(), cols, opac, scales, rots, views, projs, tanf, bg)


def test_refine_cache_follows_tensor_identity():
    from guava_renderer_amd.batch import RefineHead
    w = torch.randn(16, 32, device=DEV)
    head = RefineHead(w, torch.zeros(16, device=DEV))
    stream = torch.cuda.current_stream().cuda_stream
    a = torch.randn(1000, 32, device=DEV)
    pa = head.prepare(a, stream).clone()
    assert head.prepare(a, stream) is head._prep  # cached
    del a
    b = torch.randn(1000, 32, device=DEV)  # may reuse a's address
    pb = head.prepare(b, stream)
    torch.testing.assert_close(pb[:, 4:20], b @ w.T, rtol=1e-5, atol=1e-5)
    assert not torch.equal(pb, pa)
    b.mul_(2.0)  # in-place torch update bumps the version
    pb2 = head.prepare(b, stream)
    torch.testing.assert_close(pb2[:, 4:20], b @ w.T, rtol=1e-5, atol=1e-5)


def test_async_forward_equals_synchronous_forward(monkeypatch):
    """gsr_forward_async (binning buffer at the P x tiles bound, no R read-back) and the reference's
    synchronous gsr_forward give the same images, radii and num_rendered."""
    from guava_renderer_amd import camera, scenes
    from guava_renderer_amd.diff_gaussian_rasterization_32 import _C
    d = scenes.avatar_cloud(20000, seed=5)
    cam = camera.camera(200, 136)
    t = lambda x: torch.tensor(np.ascontiguousarray(x), device="cuda")  # noqa: E731
    empty = torch.Tensor([])
    args = (t(np.zeros(32, np.float32)), t(d["means3D"]), t(d["colors"]), t(d["opacities"]), t(d["scales"]),
            t(d["rotations"]), 1.0, empty, t(cam["viewmatrix"]), t(cam["projmatrix"]), cam["tanfovx"],
            cam["tanfovy"], 136, 200, empty, 0, t(np.zeros(3, np.float32)), False, False, False)
    Ra, ca, ra, _, bba, _, ia = _C.rasterize_gaussians(*args)
    assert isinstance(Ra, _C.PendingCount)
    monkeypatch.setattr(_C, "ASYNC_BINNING_MB", 0)
    Rs, cs, rs, _, bbs, _, is_ = _C.rasterize_gaussians(*args)
    torch.cuda.synchronize()
    assert isinstance(Rs, int) and int(Ra) == Rs and Ra == Rs and Rs > 0
    assert torch.equal(ca, cs) and torch.equal(ra, rs) and torch.equal(ia, is_)
    assert bba.numel() >= bbs.numel()


def test_binning_buffer_sizes():
    """The binning buffer autograd keeps for backward is sized to the exact instance count (as the
    reference's read-back of num_rendered does); the no-sync inference forward's P x tiles buffer
    is never saved (GaussianRasterizer_32 under no_grad keeps no context)."""
    import diff_gaussian_rasterization_32 as m
    from guava_renderer_amd import _lib, camera, scenes
    from guava_renderer_amd.diff_gaussian_rasterization_32 import _C
    d = scenes.avatar_cloud(20000, seed=5)
    cam = camera.camera(200, 136)
    t = lambda x: torch.tensor(np.ascontiguousarray(x), device="cuda")  # noqa: E731
    empty = torch.Tensor([])
    args = (t(np.zeros(32, np.float32)), t(d["means3D"]), t(d["colors"]), t(d["opacities"]), t(d["scales"]),
            t(d["rotations"]), 1.0, empty, t(cam["viewmatrix"]), t(cam["projmatrix"]), cam["tanfovx"],
            cam["tanfovy"], 136, 200, empty, 0, t(np.zeros(3, np.float32)), False, False, False)
    R, _, _, _, bb, _, _ = _C.rasterize_gaussians(*args, exact_binning=True)
    assert isinstance(R, int) and R > 0
    # the exact R: 4 B per list entry + 4 B of quad mask (the single-frame quad waves)
    assert bb.numel() == _lib.load().gsr_binning_bytes(R) <= 8 * R + 1024
    # the drop-in autograd path: the buffer saved in ctx is the exact one
    means3D = t(d["means3D"]).requires_grad_(True)
    s = m.GaussianRasterizationSettings(136, 200, cam["tanfovx"], cam["tanfovy"], t(np.zeros(32, np.float32)), 1.0,
                                        t(cam["viewmatrix"]), t(cam["projmatrix"]), 0, t(np.zeros(3, np.float32)),
                                        False, False, False)
    color, radii, _ = m.rasterize_gaussians(means3D, torch.zeros_like(means3D), empty, t(d["colors"]),
                                            t(d["opacities"]), t(d["scales"]), t(d["rotations"]), empty, s)
    saved = color.grad_fn.saved_tensors
    assert saved[9].numel() == bb.numel()  # binningBuffer
    assert isinstance(color.grad_fn.num_rendered, int) and color.grad_fn.num_rendered == R
    color.sum().backward()
    assert torch.isfinite(means3D.grad).all()
    # no graph: the no-sync path, whose count resolves to the same R
    with torch.no_grad():
        Ra, _, _, _, bba, _, _ = _C.rasterize_gaussians(*args)
    assert isinstance(Ra, _C.PendingCount) and int(Ra) == R and bba.numel() >= bb.numel()


def test_deferred_error_stays_with_its_count():
    """A prefiltered forward with a culled point (the reference's __trap) raises from its own
    num_rendered, not from a later, unrelated call that reuses its status slot."""
    from guava_renderer_amd import camera, scenes
    from guava_renderer_amd.diff_gaussian_rasterization_32 import _C
    d = scenes.random_cloud(500, seed=2)
    cam = camera.camera(64, 48)
    d["means3D"][0] = 3.0 * cam["campos"]  # behind the camera (it looks at the origin): culled
    t = lambda x: torch.tensor(np.ascontiguousarray(x), device="cuda")  # noqa: E731
    empty = torch.Tensor([])

    def args(prefiltered):
        return (t(np.zeros(32, np.float32)), t(d["means3D"]), t(d["colors"]), t(d["opacities"]), t(d["scales"]),
                t(d["rotations"]), 1.0, empty, t(cam["viewmatrix"]), t(cam["projmatrix"]), cam["tanfovx"],
                cam["tanfovy"], 48, 64, empty, 0, t(np.zeros(3, np.float32)), prefiltered, False, False)
    bad = _C.rasterize_gaussians(*args(True))[0]
    ring = next(iter(_C._RINGS.values()))
    for _ in range(ring.buf.shape[0] + 2):  # wrap the ring: every slot, the bad one included, is reused
        int(_C.rasterize_gaussians(*args(False))[0])
    with pytest.raises(RuntimeError, match="prefiltered"):
        int(bad)


def test_forward_only_batch_same_images_and_backward_refused():
    """GSR_FORWARD_ONLY (BatchRasterizer.forward(forward_only=True), the AvatarPipeline's inference
    call): preprocess skips the rows only the backward reads, binning takes the conic and mean from
    the render record -- the images, inverse depth, radii and instance count are bit-identical, and
    a backward on that workspace raises instead of reading stale rows."""
    from guava_renderer_amd import camera, scenes
    from guava_renderer_amd._lib import GsrError
    from guava_renderer_amd.batch import BatchRasterizer
    B, P, W, H = 3, 12000, 160, 128
    sc = scenes.avatar_cloud(P, seed=4)
    t = lambda x: torch.tensor(np.ascontiguousarray(x), device=DEV)  # noqa: E731
    cams = [camera.camera(W, H, yaw=y, pitch=-0.3 * y) for y in (0.0, 0.4, -0.7)]
    views = t(np.stack([c["viewmatrix"].reshape(16) for c in cams]))
    projs = t(np.stack([c["projmatrix"].reshape(16) for c in cams]))
    tanf = t(np.array([[c["tanfovx"], c["tanfovy"]] for c in cams], np.float32))
    args = [t(sc[k]) for k in ("means3D", "colors", "opacities", "scales", "rotations")]
    args += [views, projs, tanf, torch.zeros((B, 32), device=DEV)]
    r = BatchRasterizer(B, P, W, H, R_capacity=40 * P * B, device=DEV)
    ref = [x.clone() for x in r.forward(*args)]
    R_ref = r.status()[0]
    for x in r.out_color, r.out_invdepth, r.radii:
        x.fill_(7)
    got = r.forward(*args, forward_only=True)
    torch.cuda.synchronize()
    assert r.status()[0] == R_ref
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
    with pytest.raises(GsrError):
        r.backward(*args, torch.zeros((B, 32, H, W), device=DEV))
    # the C ABI refuses it too (a caller that drives the library directly, not through the mirror)
    r._fwd_only = False
    with pytest.raises(GsrError, match="FORWARD_ONLY"):
        r.backward(*args, torch.zeros((B, 32, H, W), device=DEV))
    r.forward(*args)  # a full forward makes the workspace differentiable again
    r.backward(*args, torch.zeros((B, 32, H, W), device=DEV))
    torch.cuda.synchronize()


def test_inference_path_equals_general_forward():
    """GaussianRasterizer_32 with nothing to differentiate takes _C.rasterize_inference (scratch
    arenas kept per stream, no allocator callbacks, no status copy, no autograd node): its images,
    radii and inverse depth equal _C.rasterize_gaussians' bit for bit, across calls that grow and
    reuse the scratch; with gradients on, the autograd path is still taken."""
    from diff_gaussian_rasterization_32 import GaussianRasterizationSettings, GaussianRasterizer_32
    from guava_renderer_amd.diff_gaussian_rasterization_32 import _C
    for P, W, H, seed in ((3000, 96, 80, 31), (9000, 160, 128, 32), (3000, 96, 80, 33)):
        d = make_scene("random", P, W, H, seed=seed)
        t = torch_inputs(d)
        s = GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=d["tanfovx"], tanfovy=d["tanfovy"], bg=t["bg"],
            scale_modifier=1.0, viewmatrix=t["viewmatrix"], projmatrix=t["projmatrix"], sh_degree=0,
            campos=t["campos"], prefiltered=False, debug=False, antialiasing=False)
        means2D = torch.zeros_like(t["means3D"], requires_grad=True)
        with torch.no_grad():
            col, radii, inv = GaussianRasterizer_32(s)(
                means3D=t["means3D"], means2D=means2D, opacities=t["opacities"], colors_precomp=t["colors"],
                scales=t["scales"], rotations=t["rotations"])
        assert col.grad_fn is None
        ref = _C.rasterize_gaussians(t["bg"], t["means3D"], t["colors"], t["opacities"], t["scales"],
                                     t["rotations"], 1.0, torch.Tensor([]), t["viewmatrix"], t["projmatrix"],
                                     d["tanfovx"], d["tanfovy"], H, W, torch.Tensor([]), 0, t["campos"], False,
                                     False, False)
        torch.cuda.synchronize()
        assert torch.equal(col, ref[1]) and torch.equal(radii, ref[2]) and torch.equal(inv, ref[6])
    # gradients wanted: the autograd Function (its backward runs)
    col, _, _ = GaussianRasterizer_32(s)(
        means3D=t["means3D"], means2D=means2D, opacities=t["opacities"], colors_precomp=t["colors"],
        scales=t["scales"], rotations=t["rotations"])
    assert col.grad_fn is not None
    col.sum().backward()
    assert means2D.grad is not None
