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
