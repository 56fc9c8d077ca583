"""GPU parity of the forward path (preprocess, binning/sort, render) against the CPU oracle.

Exact-exp mode (the default): every output is compared BIT-EXACTLY -- radii, tile counts,
means2D, depth, conic/opacity, the sorted per-tile lists and ranges, n_contrib, final_T, the 32
feature channels and the inverse depth.  Fast-exp mode (hardware v_exp_f32): integers exact,
colours within 1e-4 L_inf except on the rare pixels where an alpha threshold flips.
"""
import numpy as np
import pytest

from helpers import gpu_forward, make_scene, oracle_forward

pytestmark = pytest.mark.gpu


def _lib():
    from guava_renderer_amd import _lib
    return _lib


def _compare_exact(d, antialiasing=False):
    g_col, g_radii, g_inv, gs = gpu_forward(d, antialiasing=antialiasing)
    o_col, o_radii, o_inv, os_ = oracle_forward(d, exact=True, antialiasing=antialiasing)
    P = d["means3D"].shape[0]
    np.testing.assert_array_equal(g_radii, o_radii)
    vis = o_radii > 0
    np.testing.assert_array_equal(gs["tiles"], os_["tiles_touched"])
    np.testing.assert_array_equal(gs["depth"][vis], os_["depths"][vis])
    np.testing.assert_array_equal(gs["means2D"].reshape(P, 2)[vis], os_["means2D"][vis])
    np.testing.assert_array_equal(gs["conic"].reshape(P, 4)[vis], os_["conic_opacity"][vis])
    assert gs["R"] == os_["R"]
    T = os_["ranges"].shape[0]
    np.testing.assert_array_equal(gs["ranges"].reshape(T, 2), os_["ranges"])
    np.testing.assert_array_equal(gs["point_list"][:gs["R"]], os_["point_list"])
    np.testing.assert_array_equal(gs["n_contrib"], os_["n_contrib"])
    np.testing.assert_array_equal(gs["final_T"], os_["final_T"])
    np.testing.assert_array_equal(g_col, o_col)
    np.testing.assert_array_equal(g_inv, o_inv)
    return gs, os_


@pytest.mark.parametrize("kind,P,W,H", [("random", 3000, 128, 96), ("random", 10000, 256, 256),
                                        ("avatar", 20000, 200, 136)])
def test_forward_bit_exact(kind, P, W, H):
    d = make_scene(kind, P, W, H, seed=3)
    _compare_exact(d)


def test_quad_list_lengths_around_slot_and_refill_boundaries():
    """A 16x16 frame (one tile, so the single-frame quad waves walk one list): list lengths from 1
    to 28 -- the quad step takes 4 Gaussians, the step loop unrolled by the number of operand
    slots, so every exit position of the unrolled loop is taken -- and around the list refills
    (64 GSR_QUAD_RCH entries each: 192 in the product build, 256 in earlier ones): bit-exact, like
    every other forward."""
    for P in list(range(1, 29)) + [190, 192, 193, 250, 256, 257, 383, 384, 385, 512, 514]:
        d = make_scene("random", P, 16, 16, seed=100 + P)
        _compare_exact(d)


@pytest.mark.parametrize("qx,qy,seed", [(0, 0, 11), (3, 2, 12)])
def test_quad_sparse_and_dense_walks(qx, qy, seed):
    """One 16x16 tile whose list is long (~2k entries) but whose Gaussians are small and packed into
    one 4x4 quad: that quad's wave walks a dense ring, every other quad's wave finds few entries per
    192-entry refill, so its ring runs short and refills back to back (the refill loop apart from
    the step group's first refill), and every walk ends on the null padding -- bit-exact."""
    import oracle
    d = make_scene("random", 20000, 16, 16, seed=seed)
    d["scales"] = (d["scales"] * 0.15).astype(np.float32)
    st = oracle.preprocess(d["means3D"], d["scales"], d["rotations"], d["opacities"], None, d["viewmatrix"],
                           d["projmatrix"], d["image_width"], d["image_height"], d["tanfovx"], d["tanfovy"])
    m = st["means2D"].reshape(-1, 2)
    inq = (m[:, 0] >= 4 * qx) & (m[:, 0] < 4 * qx + 4) & (m[:, 1] >= 4 * qy) & (m[:, 1] < 4 * qy + 4)
    keep = inq | (np.random.default_rng(seed).random(m.shape[0]) < 0.04)
    for k in ("means3D", "colors", "opacities", "scales", "rotations"):
        d[k] = np.ascontiguousarray(d[k][keep])
    assert inq.sum() > 600 and (keep & ~inq).sum() > 300
    gs, _ = _compare_exact(d)
    assert gs["R"] > 1000


def test_forward_antialiasing_bit_exact():
    d = make_scene("random", 4000, 96, 80, seed=5)
    _compare_exact(d, antialiasing=True)


def test_forward_yaw_pitch_and_ragged_image():
    d = make_scene("avatar", 15000, 150, 101, seed=7, yaw=0.3, pitch=-0.2)
    _compare_exact(d)


def test_forward_fast_exp_tolerance():
    d = make_scene("random", 10000, 256, 256, seed=11)
    g_col, g_radii, _, gs = gpu_forward(d, numerics=_lib().numerics(fast_exp=True))
    o_col, o_radii, _, os_ = oracle_forward(d, exact=False)
    np.testing.assert_array_equal(g_radii, o_radii)
    np.testing.assert_array_equal(gs["point_list"][:gs["R"]], os_["point_list"])
    mism = (gs["n_contrib"] != os_["n_contrib"]).mean()
    assert mism <= 1e-3, mism
    same = (gs["n_contrib"] == os_["n_contrib"]).reshape(d["image_height"], d["image_width"])
    err = np.abs(g_col - o_col)[:, same]
    assert err.max() <= 1e-4, err.max()


@pytest.mark.parametrize("kind,P,W,H", [("random", 10000, 256, 256), ("avatar", 20000, 200, 136)])
def test_forward_split_bf16_tolerance(kind, P, W, H):
    """GSR_NUMERICS_SPLIT_BF16: the colour accumulation runs as four exact bf16 products per
    feature x weight on v_mfma_f32_32x32x16_bf16.  Everything the blend decides on VALU stays
    bit-exact (radii, lists, n_contrib, final_T, inverse depth); the 32 channels are within the
    north_star's 1e-4 L_inf of the oracle (bound: 3e-5 relative per product, sum of weights <= 1)."""
    d = make_scene(kind, P, W, H, seed=12)
    g_col, g_radii, g_inv, gs = gpu_forward(d, numerics=_lib().numerics(split_bf16=True))
    o_col, o_radii, o_inv, os_ = oracle_forward(d, exact=True)
    np.testing.assert_array_equal(g_radii, o_radii)
    np.testing.assert_array_equal(gs["point_list"][:gs["R"]], os_["point_list"])
    np.testing.assert_array_equal(gs["n_contrib"], os_["n_contrib"])
    np.testing.assert_array_equal(gs["final_T"], os_["final_T"])
    np.testing.assert_array_equal(g_inv, o_inv)
    err = np.abs(g_col - o_col)
    assert err.max() <= 1e-4, err.max()
    assert err.max() > 0.0  # the mode really ran (f32 accumulation is bit-exact)


def test_forward_precomputed_cov3D():
    import oracle
    d = make_scene("random", 2000, 96, 96, seed=13)
    st = oracle.preprocess(d["means3D"], d["scales"], d["rotations"], d["opacities"], None,
                           d["viewmatrix"], d["projmatrix"], 96, 96, d["tanfovx"], d["tanfovy"])
    cov = st["cov3D"]
    g_col, g_radii, _, _ = gpu_forward(d, use_cov=cov)
    o_col, o_radii, _, _ = oracle_forward(d, use_cov=True)
    np.testing.assert_array_equal(g_radii, o_radii)
    np.testing.assert_array_equal(g_col, o_col)


@pytest.mark.parametrize("kind,P,W,H", [("random", 3000, 128, 96), ("avatar", 20000, 200, 136)])
def test_render_counters_match_oracle(kind, P, W, H):
    """The instrumented render kernel (gsr_render_counters) gives the same image and counts exactly
    the pairs the reference's per-pixel loop visits and blends."""
    import oracle
    from guava_renderer_amd.batch import render_counters
    d = make_scene(kind, P, W, H, seed=3)
    res = {}
    cnt = render_counters(lambda: res.update(out=gpu_forward(d)))
    g_col, g_radii, g_inv, gs = res["out"]
    o_col, _, _, os_ = oracle_forward(d, exact=True)
    np.testing.assert_array_equal(g_col, o_col)
    visited, contrib = oracle.render_counts(os_, W, H)
    assert cnt["pairs_evaluated"] == visited
    assert cnt["pairs_contributing"] == contrib
    assert cnt["list_entries"] == gs["R"]
    # lane-pairs blended: 64 per survivor in the strip layout
    assert contrib <= cnt["strip_pairs_blended"] * 64
    # survivors are taken two per k-step, an odd round tail pads with the null Gaussian
    assert cnt["strip_pairs_blended"] <= 2 * cnt["mfma_ksteps"] <= cnt["strip_pairs_blended"] + cnt["gaussians_staged"]


def test_strip_work_list():
    """k_strip_count / k_strip_place: survivors per 64-pixel strip equal the popcount of that strip's
    bit over the tile's list, and the strip work list holds every strip of every non-empty tile
    exactly once, tile-major (GSR_STRIP_ORDER default): a tile's 4 strips consecutive, tiles in
    non-increasing order of their longest strip up to the 4-buckets-per-octave granularity."""
    d = make_scene("avatar", 20000, 200, 136, seed=3)
    _, _, _, gs = gpu_forward(d)
    T = gs["ranges"].size // 2
    rg = gs["ranges"].reshape(T, 2)
    cnt = gs["strip_cnt"].reshape(T, 4)
    for t in range(T):
        m = gs["smask"][rg[t, 0]:rg[t, 1]]
        np.testing.assert_array_equal(cnt[t], [(m >> s & 1).sum() for s in range(4)])
    nonempty = np.nonzero(gs["tile_count"])[0]
    n = 4 * len(nonempty)
    lst = gs["strip_list"][:n]
    assert sorted(lst.tolist()) == sorted((4 * nonempty[:, None] + np.arange(4)).reshape(-1).tolist())

    def bucket(c):
        if c == 0:
            return 128
        e = int(c).bit_length() - 1
        sub = (c >> (e - 2)) & 3 if e >= 2 else (c << (2 - e)) & 3
        return 127 - (4 * e + sub)
    groups = lst.reshape(-1, 4)
    assert (groups >> 2 == (groups[:, :1] >> 2)).all() and ((groups & 3) == np.arange(4)).all()
    # one frame: one longest-first list (batches of 2+ frames use per-XCD segments, each
    # longest-first: queue_item map 2; every batch test's bit-exact frames cover that walk)
    b = [bucket(int(cnt[x >> 2].max())) for x in groups[:, 0]]
    assert all(b[i] <= b[i + 1] for i in range(len(b) - 1))


def test_refine_epilogue_matches_conv():
    """The fused StyleUNet conv_body_first + leaky ReLU (styleunet.py:110,178) equals torch's conv2d
    on the full render within 1e-5 of scale (the conv is applied to each Gaussian's features before
    compositing -- an exact algebraic reassociation, rounded differently); the kept raw channels
    are bit-identical to the plain render and the others are not written."""
    import torch
    import torch.nn.functional as F
    from guava_renderer_amd.batch import BatchRasterizer, RefineHead
    from guava_renderer_amd import scenes
    dev = "cuda:0"
    B, P, W, H = 3, 6000, 96, 80  # ragged image: partial tiles on both axes
    sc = scenes.random_cloud(P, seed=3)
    t = lambda x: torch.tensor(np.ascontiguousarray(x), device=dev)  # noqa: E731
    cams = scenes.frame_cameras(B, W, H, seed=7)
    views = t(np.stack([c["viewmatrix"].reshape(16) for c in cams]))
    projs = t(np.stack([c["projmatrix"].reshape(16) for c in cams]))
    tanf = t(np.array([[c["tanfovx"], c["tanfovy"]] for c in cams], np.float32))
    bgs = t(np.random.default_rng(0).normal(size=(B, 32)).astype(np.float32))
    args = (t(sc["means3D"]), t(sc["colors"]), t(sc["opacities"]), t(sc["scales"]), t(sc["rotations"]),
            views, projs, tanf, bgs)
    r = BatchRasterizer(B, P, W, H, device=dev)
    full = r.forward(*args)[0].clone()
    rng = np.random.default_rng(1)
    head = RefineHead(t(rng.normal(0, 0.2, (16, 32)).astype(np.float32)),
                      t(rng.normal(0, 0.1, 16).astype(np.float32)), keep_channels=4)
    r.out_color.fill_(12345.0)
    col = r.forward(*args, refine=head)[0]
    torch.cuda.synchronize()
    assert torch.equal(col[:, :4], full[:, :4])
    assert (col[:, 4:] == 12345.0).all()
    ref = F.leaky_relu(F.conv2d(full, head.weight[:, :, None, None], head.bias), 0.2)
    err = (head.out - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, err


def _batch_vs_oracle(kind, P, W, H, seed, antialiasing=False, yaw=(0.0, 0.25), counters=False):
    """Frames through the batched entry (B > 1: the throughput render kernel, queue map 2) against
    the oracle, per frame, bit-exactly."""
    import torch
    from guava_renderer_amd import camera, scenes
    from guava_renderer_amd.batch import BatchRasterizer, render_counters
    import oracle
    sc = scenes.random_cloud(P, seed) if kind == "random" else scenes.avatar_cloud(P, seed)
    cams = [camera.camera(W, H, yaw=y, pitch=-0.5 * y) for y in yaw]
    B = len(cams)
    t = lambda x: torch.tensor(np.ascontiguousarray(x), device="cuda")  # noqa: E731
    args = [t(sc[k]) for k in ("means3D", "colors", "opacities", "scales", "rotations")]
    views = t(np.stack([c["viewmatrix"].reshape(16) for c in cams]))
    projs = t(np.stack([c["projmatrix"].reshape(16) for c in cams]))
    tanf = t(np.array([[c["tanfovx"], c["tanfovy"]] for c in cams], np.float32))
    r = BatchRasterizer(B, P, W, H, R_capacity=40 * P * B, device="cuda")
    res = {}
    fwd = lambda: res.update(out=r.forward(*args, views, projs, tanf, torch.zeros((B, 32), device="cuda"),  # noqa: E731
                                           antialiasing=antialiasing))
    cnt = render_counters(fwd) if counters else (fwd(), None)[1]
    col, inv, radii = (x.cpu().numpy() for x in res["out"])
    assert not r.status()[1]
    visited = contrib = 0
    for f, c in enumerate(cams):
        o_col, o_radii, o_inv, os_ = oracle.forward(sc["means3D"], sc["colors"], sc["opacities"], sc["scales"],
                                                    sc["rotations"], None, c["viewmatrix"], c["projmatrix"], W, H,
                                                    c["tanfovx"], c["tanfovy"], np.zeros(32, np.float32),
                                                    antialiasing=antialiasing)
        np.testing.assert_array_equal(radii[f], o_radii)
        np.testing.assert_array_equal(col[f], o_col)
        np.testing.assert_array_equal(inv[f], o_inv.reshape(H, W))
        if counters:
            v, k = oracle.render_counts(os_, W, H)
            visited += v
            contrib += k
    if counters:
        assert cnt["pairs_evaluated"] == visited and cnt["pairs_contributing"] == contrib
        assert contrib <= cnt["strip_pairs_blended"] * 64


@pytest.mark.parametrize("kind,P,W,H", [("random", 10000, 256, 256), ("avatar", 20000, 200, 136),
                                        ("random", 3000, 96, 80)])
def test_batch_render_bit_exact(kind, P, W, H):
    _batch_vs_oracle(kind, P, W, H, seed=21)


def test_batch_render_antialiasing_and_counters():
    _batch_vs_oracle("avatar", 15000, 150, 101, seed=22, antialiasing=True, yaw=(0.3, -0.2, 0.0), counters=True)


def test_batch_render_long_lists():
    """Dense splats: strips with hundreds of survivors (several 64-entry index chunks per strip,
    the DMA ring wrapping many times, odd survivor counts)."""
    _batch_vs_oracle("random", 40000, 64, 64, seed=23)
