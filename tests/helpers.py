"""Shared test helpers: scene construction, GPU calls through the drop-in API, oracle calls and
scratch-arena decoding (mirrors carve_geom/carve_image/carve_bin in
guava_renderer_amd/csrc/capi.hip -- keep in sync)."""
import numpy as np

C = 32


def _align(x):
    return (x + 255) & ~255


def _carve(spec):
    off = 0
    out = {}
    for name, dtype, count in spec:
        off = _align(off)
        out[name] = (off, np.dtype(dtype), count)
        off += np.dtype(dtype).itemsize * count
    return out


def _nb(P):
    nb = 64
    while nb < P // 8 and nb < (1 << 20):
        nb <<= 1
    return nb


def geom_layout(P, W, H):
    nblk = (P + 255) // 256
    T = ((W + 15) // 16) * ((H + 15) // 16)
    NB = _nb(P)
    chunk = 1024 if T > 1024 else 256  # make_dims: count-table rows
    nchunk = (P + chunk - 1) // chunk
    return _carve([("ctrl", np.uint32, 9216 + 8), ("depth", np.float32, P), ("invdepth", np.float32, P),
                   ("radii", np.int32, P), ("means2D", np.float32, 2 * P), ("cov3D", np.float32, 6 * P),
                   ("conic", np.float32, 4 * P), ("rect", np.uint32, 2 * P), ("rrec", np.float32, 8 * P),
                   ("tiles", np.uint32, P), ("blocksums", np.uint32, nblk + 1), ("blockkey", np.uint32, 2 * nblk), ("bslot", np.uint32, P),
                   ("bstart", np.uint32, NB + 1), ("skey", np.uint64, P), ("big", np.uint32, NB),
                   ("order", np.uint32, P), ("table", np.uint32, nchunk * T)])


def image_layout(W, H):
    T = ((W + 15) // 16) * ((H + 15) // 16)
    return _carve([("final_T", np.float32, W * H), ("n_contrib", np.uint32, W * H),
                   ("ranges", np.uint32, 2 * T), ("tile_count", np.uint32, T), ("work_list", np.uint32, T),
                   ("lpt_hist", np.uint32, 34), ("strip_cnt", np.uint32, 4 * T),
                   ("strip_list", np.uint32, 4 * T), ("strip_hist", np.uint32, 8 * 129)])


def bin_layout(R):
    n = max(R, 1)
    return _carve([("point_list", np.uint32, n)])


def decode(buf_np, layout):
    out = {}
    for name, (off, dt, count) in layout.items():
        out[name] = np.frombuffer(buf_np[off:off + dt.itemsize * count].tobytes(), dtype=dt).copy()
    return out


def make_scene(kind="random", P=2000, W=128, H=96, seed=0, yaw=0.0, pitch=0.0):
    from guava_renderer_amd import camera, scenes
    if kind == "random":
        d = scenes.random_cloud(P, seed)
    else:
        d = scenes.avatar_cloud(P, seed)
    cam = camera.camera(W, H, yaw=yaw, pitch=pitch)
    d.update(cam)
    d["bg"] = np.zeros(C, np.float32)
    return d


def oracle_forward(d, exact=True, antialiasing=False, use_cov=False):
    import oracle
    cov = None
    if use_cov:
        st = oracle.preprocess(d["means3D"], d["scales"], d["rotations"], d["opacities"], None,
                               d["viewmatrix"], d["projmatrix"], d["image_width"], d["image_height"],
                               d["tanfovx"], d["tanfovy"])
        cov = st["cov3D"]
    color, radii, invd, st = oracle.forward(
        d["means3D"], d["colors"], d["opacities"], None if use_cov else d["scales"],
        None if use_cov else d["rotations"], cov, d["viewmatrix"], d["projmatrix"],
        d["image_width"], d["image_height"], d["tanfovx"], d["tanfovy"], d["bg"],
        antialiasing=antialiasing, exact_exp=exact)
    return color, radii, invd, st


def torch_inputs(d, device="cuda", requires_grad=False):
    import torch
    t = {}
    for k in ("means3D", "colors", "opacities", "scales", "rotations"):
        t[k] = torch.tensor(d[k], device=device, requires_grad=requires_grad)
    t["viewmatrix"] = torch.tensor(d["viewmatrix"], device=device)
    t["projmatrix"] = torch.tensor(d["projmatrix"], device=device)
    t["campos"] = torch.tensor(d["campos"], device=device)
    t["bg"] = torch.tensor(d["bg"], device=device)
    return t


def gpu_forward(d, antialiasing=False, use_cov=None, debug=False, numerics=0):
    """Runs _C.rasterize_gaussians; returns numpy outputs plus decoded scratch state."""
    import torch
    from guava_renderer_amd.diff_gaussian_rasterization_32 import _C
    t = torch_inputs(d)
    empty = torch.Tensor([])
    cov = empty if use_cov is None else torch.tensor(use_cov, device="cuda")
    scales = t["scales"] if use_cov is None else empty
    rots = t["rotations"] if use_cov is None else empty
    R, color, radii, gb, bb, ib, invd = _C.rasterize_gaussians(
        t["bg"], t["means3D"], t["colors"], t["opacities"], scales, rots, 1.0, cov,
        t["viewmatrix"], t["projmatrix"], d["tanfovx"], d["tanfovy"], d["image_height"],
        d["image_width"], empty, 0, t["campos"], False, antialiasing, debug, numerics=numerics)
    torch.cuda.synchronize()
    P = d["means3D"].shape[0]
    W, H = d["image_width"], d["image_height"]
    st = {}
    st.update(decode(gb.cpu().numpy(), geom_layout(P, W, H)))
    st.update(decode(ib.cpu().numpy(), image_layout(W, H)))
    # the binning buffer is carved for its capacity: R after the synchronous read-back, the P x tiles
    # bound on the no-sync path
    from guava_renderer_amd import _lib
    L = _lib.load()
    cap = int(R) if bb.numel() == L.gsr_binning_bytes(int(R)) else L.gsr_forward_async_bound(P, W, H)
    st.update(decode(bb.cpu().numpy(), bin_layout(cap)))
    st["smask"] = st["point_list"] >> 28           # entries: index | strip mask << 28
    st["point_list"] = st["point_list"] & 0x0FFFFFFF
    st["R"] = R
    return color.cpu().numpy(), radii.cpu().numpy(), invd.cpu().numpy(), st


GRAD_SCALE_TOL = 1e-4   # |a - b| <= 1e-4 * max|b| over the whole tensor
GRAD_ELEM_TOL = 1e-3    # |a - b| <= 1e-3 * |b| on every element with |b| >= GRAD_ELEM_FLOOR * max|b|
GRAD_ELEM_FLOOR = 1e-3


NOISE_FACTOR = 1.5      # per-element bound relative to the reference algorithm's own f32 reordering noise
                        # (worst measured GPU / reordering ratio 1.26)


def grad_check(name, a, b, scale_tol=GRAD_SCALE_TOL, elem_tol=GRAD_ELEM_TOL, floor=GRAD_ELEM_FLOOR,
               noise=None, p999_tol=None):
    """Gradient parity, two ways: against the tensor's scale (the per-Gaussian atomics of the
    reference, backward.cu:593-635, reassociate freely) and per element -- a Gaussian with a small but
    not negligible gradient must be right too: relative error <= elem_tol on every element with
    |g| >= floor * max|g|.  `noise`: the same oracle gradient accumulated in another order
    (oracle.backward(reverse_order=True)); the closed-form backward amplifies f32 reassociation on
    ill-conditioned elements (the 2x2 conic inverse, computeCov2DCUDA, backward.cu:147-326), so the
    per-element bound is max(elem_tol, NOISE_FACTOR x the reference's own reordering error), and the
    99.9th percentile must stay within p999_tol (default elem_tol / 10).  Prints both distributions."""
    a = np.asarray(a, np.float64).reshape(-1)
    b = np.asarray(b, np.float64).reshape(-1)
    assert a.shape == b.shape, (name, a.shape, b.shape)
    m = float(np.abs(b).max()) if b.size else 0.0
    if m == 0.0:
        assert np.abs(a).max(initial=0.0) == 0.0, name
        return
    err_scale = float(np.abs(a - b).max()) / m
    big = np.abs(b) >= floor * m
    rel = np.abs(a - b)[big] / np.abs(b)[big]
    p999 = float(np.percentile(rel, 99.9)) if rel.size else 0.0
    limit = elem_tol
    msg = ""
    if noise is not None:
        nz = np.asarray(noise, np.float64).reshape(-1)
        rel_n = np.abs(nz - b)[big] / np.abs(b)[big]
        limit = max(elem_tol, NOISE_FACTOR * float(rel_n.max(initial=0.0)))
        msg = (f"; reference reordered: max {rel_n.max(initial=0.0):.3g}, "
               f"p99.9 {float(np.percentile(rel_n, 99.9)) if rel_n.size else 0.0:.3g}")
    print(f"  {name}: {err_scale:.3g} of scale; elementwise over {int(big.sum())} |g| >= {floor:g} max: "
          f"max {rel.max(initial=0.0):.3g}, p99.9 {p999:.3g}{msg}")
    assert err_scale <= scale_tol, f"{name}: {err_scale:.3g} of scale"
    assert rel.max(initial=0.0) <= limit, f"{name}: element rel err {rel.max():.3g} > {limit:.3g} (p99.9 {p999:.3g})"
    p999_tol = elem_tol / 10 if p999_tol is None else p999_tol
    assert p999 <= p999_tol, f"{name}: element rel err p99.9 {p999:.3g} > {p999_tol:.3g}"
