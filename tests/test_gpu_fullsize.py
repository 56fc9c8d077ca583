"""GPU parity at BASELINE.json's full sizes.

* One frame of config 2 (the 100k-Gaussian avatar at 512x512) and one of config 5 (300k Gaussians
  at 1024x1024) rendered through the batched entry (gsr_forward_batch, the bench's path) and
  compared BIT-EXACTLY with the CPU oracle: colours, inverse depth, radii.
* Size-independent invariants over a whole 32-frame config-2 batch (the bench's workload):
  - every frame of the batch equals that frame rendered alone through the reference API
    (_C.rasterize_gaussians) -- batching changes nothing;
  - with every feature channel set to 1 and a zero background, each pixel's channel equals its
    accumulated opacity 1 - final_T (sum of the blend weights) to float rounding;
  - 0 <= final_T <= 1 and the inverse depth is non-negative.
"""
import numpy as np
import pytest
import torch

from helpers import decode, image_layout, oracle_forward

pytestmark = pytest.mark.gpu


def _batch_render(sc, cams, colors=None, split_bf16=False):
    from guava_renderer_amd import _lib
    from guava_renderer_amd.batch import BatchRasterizer
    dev = torch.device("cuda")
    t = lambda x: torch.tensor(np.ascontiguousarray(x), device=dev)  # noqa: E731
    B = len(cams)
    W, H = cams[0]["image_width"], cams[0]["image_height"]
    P = sc["means3D"].shape[0]
    views = t(np.stack([c["viewmatrix"].reshape(16) for c in cams]))
    projs = t(np.stack([c["projmatrix"].reshape(16) for c in cams]))
    tanf = t(np.array([[c["tanfovx"], c["tanfovy"]] for c in cams], np.float32))
    r = BatchRasterizer(B, P, W, H, R_capacity=24 * P * B, device=dev,
                        numerics=_lib.numerics(split_bf16=split_bf16))
    col, inv, radii = r.forward(t(sc["means3D"]), t(sc["colors"] if colors is None else colors),
                                t(sc["opacities"]), t(sc["scales"]), t(sc["rotations"]), views, projs, tanf,
                                torch.zeros((B, 32), device=dev))
    torch.cuda.synchronize()
    R, ovf = r.status()
    assert not ovf
    return r, col.cpu().numpy(), inv.cpu().numpy(), radii.cpu().numpy()


@pytest.mark.parametrize("P,W,gpt", [(100000, 512, 1), (300000, 1024, 3)])
def test_full_size_frame_bit_exact(P, W, gpt):
    from guava_renderer_amd import scenes
    sc = scenes.avatar_cloud(P, seed=0, gaussians_per_texel=gpt)
    cam = scenes.frame_cameras(2, W, W, seed=1000)[1]  # an orbit camera (yaw/pitch != 0)
    _, col, inv, radii = _batch_render(sc, [cam])
    import oracle
    oracle.set_threads(8)
    d = dict(sc, **cam, bg=np.zeros(32, np.float32))
    o_col, o_radii, o_inv, _ = oracle_forward(d, exact=True)
    np.testing.assert_array_equal(radii[0], o_radii)
    np.testing.assert_array_equal(col[0], o_col)
    np.testing.assert_array_equal(inv[0].reshape(o_inv.shape), o_inv)


def test_full_size_frame_split_bf16():
    """The bench's colour-accumulation mode at config-2 size: colour within the north_star's 1e-4
    L_inf of the oracle, inverse depth and radii bit-exact."""
    from guava_renderer_amd import scenes
    sc = scenes.avatar_cloud(100000, seed=0)
    cam = scenes.frame_cameras(2, 512, 512, seed=1000)[1]
    _, col, inv, radii = _batch_render(sc, [cam], split_bf16=True)
    import oracle
    oracle.set_threads(8)
    d = dict(sc, **cam, bg=np.zeros(32, np.float32))
    o_col, o_radii, o_inv, _ = oracle_forward(d, exact=True)
    np.testing.assert_array_equal(radii[0], o_radii)
    np.testing.assert_array_equal(inv[0].reshape(o_inv.shape), o_inv)
    err = np.abs(col[0] - o_col)
    print("split-bf16 colour L_inf vs oracle:", err.max(), "RGB:", err[:3].max())
    assert err.max() <= 1e-4, err.max()


def test_split_bf16_per_frame_colors():
    """Split-bf16 with per-frame feature tables ([B, P, 32], split inside render_fwd) against the
    shared-table path (pre-split once per launch): the same packed words, so bit-identical frames;
    and within 1e-4 of the exact (f32 MFMA) render."""
    from guava_renderer_amd import scenes
    sc = scenes.avatar_cloud(20000, seed=3)
    cams = scenes.frame_cameras(2, 256, 256, seed=1000)
    per_frame = np.ascontiguousarray(np.broadcast_to(sc["colors"], (2,) + sc["colors"].shape))
    _, col_pf, inv_pf, _ = _batch_render(sc, cams, colors=per_frame, split_bf16=True)
    _, col_sh, inv_sh, _ = _batch_render(sc, cams, split_bf16=True)
    _, col_ex, inv_ex, _ = _batch_render(sc, cams)
    np.testing.assert_array_equal(col_pf, col_sh)
    np.testing.assert_array_equal(inv_pf, inv_ex)
    err = np.abs(col_sh - col_ex).max()
    assert 0.0 < err <= 1e-4, err


def test_full_batch_invariants():
    from guava_renderer_amd import scenes
    from guava_renderer_amd.diff_gaussian_rasterization_32 import _C
    sc = scenes.avatar_cloud(100000, seed=0)
    cams = scenes.frame_cameras(32, 512, 512, seed=1000)
    ones = np.ones_like(sc["colors"])
    r, col, inv, _ = _batch_render(sc, cams, colors=ones)
    acc = col[:, 0]  # every channel equals the accumulated opacity when all features are 1
    for ch in (1, 17, 31):
        np.testing.assert_array_equal(col[:, ch], acc)
    assert (acc >= 0).all() and (acc <= 1.0 + 1e-6).all()
    assert (inv >= 0).all()
    # frames 0, 13 and 31 equal single-frame renders through the reference API
    dev = torch.device("cuda")
    for k in (0, 13, 31):
        c = cams[k]
        t = lambda x: torch.tensor(np.ascontiguousarray(x), device=dev)  # noqa: E731
        empty = torch.Tensor([])
        _, col1, _, _, _, ib, inv1 = _C.rasterize_gaussians(
            torch.zeros(32, device=dev), t(sc["means3D"]), t(ones), t(sc["opacities"]), t(sc["scales"]),
            t(sc["rotations"]), 1.0, empty, t(c["viewmatrix"]), t(c["projmatrix"]), c["tanfovx"], c["tanfovy"],
            512, 512, empty, 0, t(c["campos"]), False, False, False)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(col1.cpu().numpy(), col[k])
        np.testing.assert_array_equal(inv1.cpu().numpy().reshape(inv[k].shape), inv[k])
        final_T = decode(ib.cpu().numpy(), image_layout(512, 512))["final_T"].reshape(512, 512)
        assert (final_T >= 0).all() and (final_T <= 1).all()
        np.testing.assert_allclose(acc[k], 1.0 - final_T, atol=2e-5)


def test_block_affine_queue_segments():
    """Batches (B >= 2) deal the strips over the eight per-XCD queues by 4x4-tile block
    (queue_item map 2): the control words hold each queue's segment of the strip list, and the
    segments tile the non-empty tiles exactly (start = exclusive sum of the counts); the frames
    themselves are pinned bit-exactly by the other batch tests."""
    from guava_renderer_amd import scenes
    sc = scenes.avatar_cloud(20000, seed=3)
    cams = scenes.frame_cameras(3, 256, 256, seed=1000)
    r, _, _, _ = _batch_render(sc, cams)
    ctrl = r.workspace[:4 * 64].view(torch.int32).cpu().numpy()
    ne, qstart, qcount = int(ctrl[6]), ctrl[16:24], ctrl[24:32]
    assert ne > 0 and int(qcount.sum()) == ne
    np.testing.assert_array_equal(qstart, np.concatenate([[0], np.cumsum(qcount)[:-1]]))
    assert (qcount > 0).sum() >= 4  # the blocks spread over the queues

