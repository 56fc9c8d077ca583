"""ctypes front-end of the CPU oracle (oracle/gsr_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker.  The product path
(guava_renderer_amd, libgsr.so) never imports this module.

Mirrors the reference driver CudaRasterizer::Rasterizer::forward/backward
(/root/reference/submodules/diff-gaussian-rasterization-32/cuda_rasterizer/
rasterizer_impl.cu:198-341, :345-450) on numpy arrays.
"""
import ctypes
import os
import subprocess

import numpy as np

C = 32
BLOCK = 16
_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "lib", "libgsr_oracle.so")
_lib = None

_f = ctypes.POINTER(ctypes.c_float)
_i = ctypes.POINTER(ctypes.c_int)
_u32 = ctypes.POINTER(ctypes.c_uint32)
_u64 = ctypes.POINTER(ctypes.c_uint64)
_u8 = ctypes.POINTER(ctypes.c_uint8)


def build():
    """Compile the oracle (make -C oracle)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.gsro_expf.restype = ctypes.c_float
        L.gsro_expf.argtypes = [ctypes.c_float]
        L.gsro_blend_alpha.restype = ctypes.c_float
        L.gsro_blend_alpha.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_int]
        L.gsro_blend_G.restype = ctypes.c_float
        L.gsro_blend_G.argtypes = [ctypes.c_float, ctypes.c_int]
        L.gsro_mark_visible.argtypes = [ctypes.c_int, _f, _f, _f, _u8]
        L.gsro_preprocess.restype = ctypes.c_int
        L.gsro_preprocess.argtypes = [ctypes.c_int, _f, _f, ctypes.c_float, _f, _f, _f, _f, _f,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                      ctypes.c_int, ctypes.c_int, _i, _f, _f, _f, _f, _u32]
        L.gsro_bin.restype = ctypes.c_int64
        L.gsro_bin.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _i, _f, _f, _u32, _u32,
                               _u32, _u64, _u32, ctypes.c_int64]
        L.gsro_render.argtypes = [ctypes.c_int, ctypes.c_int, _u32, _u32, _f, _f, _f, _f, _f,
                                  ctypes.c_int, _f, _f, _f, _u32]
        L.gsro_render_counts.argtypes = [ctypes.c_int, ctypes.c_int, _u32, _u32, _f, _f, ctypes.c_int,
                                         _u64]
        L.gsro_render_decision_flips.restype = ctypes.c_uint64
        L.gsro_render_decision_flips.argtypes = [ctypes.c_int, ctypes.c_int, _u32, _u32, _f, _f, _u8]
        L.gsro_set_backward_order.argtypes = [ctypes.c_int]
        L.gsro_render_decision_flips_modes.restype = ctypes.c_uint64
        L.gsro_render_decision_flips_modes.argtypes = [ctypes.c_int, ctypes.c_int, _u32, _u32, _f, _f,
                                                       ctypes.c_int, ctypes.c_int, _u8]
        L.gsro_render_backward.argtypes = [ctypes.c_int, ctypes.c_int, _u32, _u32, _f, _f, _f, _f,
                                           _f, _f, _u32, _f, _f, ctypes.c_int, _f, _f, _f, _f, _f]
        L.gsro_preprocess_backward.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _f, _i, _f,
                                               ctypes.c_float, _f, _f, _f, _f, _f, ctypes.c_float,
                                               ctypes.c_float, _f, _f, _f, ctypes.c_int, _f, _f, _f,
                                               _f, _f]
        L.gsro_set_threads.argtypes = [ctypes.c_int]
        L.gsro_get_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a, t):
    if a is None:
        return ctypes.cast(None, t)
    return a.ctypes.data_as(t)


def _f32(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float32)


def set_threads(n):
    lib().gsro_set_threads(int(n))


def get_threads():
    return lib().gsro_get_threads()


def expf(x):
    x = np.asarray(x, dtype=np.float32).ravel()
    return np.array([lib().gsro_expf(float(v)) for v in x], dtype=np.float32)


def blend_alpha(o, x):
    """min(0.99, o exp(x)) as the blend evaluates it (exact mode)."""
    x = np.asarray(x, dtype=np.float32).ravel()
    return np.array([lib().gsro_blend_alpha(float(o), float(v), 1) for v in x], dtype=np.float32)


def blend_G(x):
    x = np.asarray(x, dtype=np.float32).ravel()
    return np.array([lib().gsro_blend_G(float(v), 1) for v in x], dtype=np.float32)


def grid_dims(W, H):
    return (W + BLOCK - 1) // BLOCK, (H + BLOCK - 1) // BLOCK


def mark_visible(means3D, view, proj):
    means3D = _f32(means3D)
    P = means3D.shape[0]
    out = np.zeros(P, np.uint8)
    lib().gsro_mark_visible(P, _p(means3D, _f), _p(_f32(view), _f), _p(_f32(proj), _f), _p(out, _u8))
    return out.astype(bool)


def preprocess(means3D, scales, rotations, opacities, cov3D_precomp, view, proj, W, H, tanx, tany,
               scale_modifier=1.0, prefiltered=False, antialiasing=False):
    means3D = _f32(means3D)
    P = means3D.shape[0]
    st = dict(
        radii=np.zeros(P, np.int32), means2D=np.zeros((P, 2), np.float32),
        depths=np.zeros(P, np.float32), cov3D=np.zeros((P, 6), np.float32),
        conic_opacity=np.zeros((P, 4), np.float32), tiles_touched=np.zeros(P, np.uint32))
    scales = _f32(scales)
    rotations = _f32(rotations)
    cov3D_precomp = _f32(cov3D_precomp)
    opac = _f32(opacities).reshape(-1)
    rc = lib().gsro_preprocess(
        P, _p(means3D, _f), _p(scales, _f), float(scale_modifier), _p(rotations, _f), _p(opac, _f),
        _p(cov3D_precomp, _f), _p(_f32(view), _f), _p(_f32(proj), _f), int(W), int(H),
        float(tanx), float(tany), int(bool(prefiltered)), int(bool(antialiasing)),
        _p(st["radii"], _i), _p(st["means2D"], _f), _p(st["depths"], _f), _p(st["cov3D"], _f),
        _p(st["conic_opacity"], _f), _p(st["tiles_touched"], _u32))
    if rc != 0:
        raise RuntimeError("prefiltered is set but a point was culled")
    if cov3D_precomp is not None:
        st["cov3D"] = cov3D_precomp.reshape(P, 6).copy()
    return st


def bin_and_sort(st, W, H):
    P = st["radii"].shape[0]
    gx, gy = grid_dims(W, H)
    T = gx * gy
    R = int(st["tiles_touched"].astype(np.uint64).sum())
    offs = np.zeros(P, np.uint32)
    pl = np.zeros(max(R, 1), np.uint32)
    keys = np.zeros(max(R, 1), np.uint64)
    ranges = np.zeros((T, 2), np.uint32)
    r = lib().gsro_bin(P, int(W), int(H), _p(st["radii"], _i), _p(st["means2D"], _f),
                       _p(st["depths"], _f), _p(st["tiles_touched"], _u32), _p(offs, _u32),
                       _p(pl, _u32), _p(keys, _u64), _p(ranges, _u32), R)
    assert r == R, (r, R)
    st.update(point_offsets=offs, point_list=pl[:R], point_keys=keys[:R], ranges=ranges, R=R)
    return st


LITERAL = "literal"


def _mode(exact_exp):
    """Blend arithmetic mode of the C oracle (gsr_oracle.c, "Blend arithmetic modes"): True -> 1 (the
    restatement the GPU reproduces bit for bit), False -> 0 (the same with libm expf), "literal" -> 2
    (the reference's expressions as written, forward.cu:352-391 / backward.cu:564-568, libm expf)."""
    if exact_exp == LITERAL:
        return 2
    return int(bool(exact_exp))


def render(st, colors, bg, W, H, exact_exp=True):
    colors = _f32(colors)
    HW = W * H
    out = np.zeros((C, H, W), np.float32)
    invd = np.zeros((1, H, W), np.float32)
    fT = np.zeros(HW, np.float32)
    nc = np.zeros(HW, np.uint32)
    pl = st["point_list"] if st["R"] > 0 else np.zeros(1, np.uint32)
    lib().gsro_render(int(W), int(H), _p(st["ranges"], _u32), _p(pl, _u32),
                      _p(st["means2D"], _f), _p(colors, _f), _p(st["conic_opacity"], _f),
                      _p(st["depths"], _f), _p(_f32(bg), _f), _mode(exact_exp),
                      _p(out, _f), _p(invd, _f), _p(fT, _f), _p(nc, _u32))
    st.update(final_T=fT, n_contrib=nc)
    return out, invd


def render_counts(st, W, H, exact_exp=True):
    """(pairs visited, pairs contributing) of the per-pixel blend loop (forward.cu:336-381)."""
    out = np.zeros(2, np.uint64)
    pl = st["point_list"] if st["R"] > 0 else np.zeros(1, np.uint32)
    lib().gsro_render_counts(int(W), int(H), _p(st["ranges"], _u32), _p(pl, _u32),
                             _p(st["means2D"], _f), _p(st["conic_opacity"], _f), _mode(exact_exp),
                             _p(out, _u64))
    return int(out[0]), int(out[1])


def decision_flips(st, W, H, against=False):
    """Pixels whose blend takes or stops differently with the restatement's arithmetic (the GPU's)
    and with `against` (False: the same arithmetic with libm expf; "literal": the reference's
    expressions as written, gsro_render_decision_flips_modes): bool [H, W]."""
    flags = np.zeros(W * H, np.uint8)
    pl = st["point_list"] if st["R"] > 0 else np.zeros(1, np.uint32)
    lib().gsro_render_decision_flips_modes(int(W), int(H), _p(st["ranges"], _u32), _p(pl, _u32),
                                           _p(st["means2D"], _f), _p(st["conic_opacity"], _f), 1,
                                           _mode(against), _p(flags, _u8))
    return flags.reshape(H, W).astype(bool)


def forward(means3D, colors, opacities, scales, rotations, cov3D_precomp, view, proj, W, H, tanx,
            tany, bg, scale_modifier=1.0, prefiltered=False, antialiasing=False, exact_exp=True):
    """Full forward (rasterizer_impl.cu:198-341). Returns (color[C,H,W], radii[P], invdepth[1,H,W], state)."""
    st = preprocess(means3D, scales, rotations, opacities, cov3D_precomp, view, proj, W, H, tanx,
                    tany, scale_modifier, prefiltered, antialiasing)
    bin_and_sort(st, W, H)
    color, invd = render(st, colors, bg, W, H, exact_exp)
    return color, st["radii"].copy(), invd, st


def backward(st, means3D, colors, opacities, scales, rotations, cov3D_precomp, view, proj, W, H,
             tanx, tany, bg, dL_dcolor, dL_dinvdepth=None, scale_modifier=1.0, antialiasing=False,
             exact_exp=True, reverse_order=False):
    """Full backward (rasterizer_impl.cu:345-450).  reverse_order: the per-Gaussian sums accumulated
    over tiles and pixels in reverse (gsro_set_backward_order; the f32 reassociation noise floor).
    Returns the 8 grads in _C order:
    (dL_dmeans2D[P,3], dL_dcolors[P,C], dL_dopacity[P,1], dL_dmeans3D[P,3], dL_dcov3D[P,6],
     dL_dsh[P,0,3], dL_dscales[P,3], dL_drotations[P,4])."""
    means3D = _f32(means3D)
    P = means3D.shape[0]
    g_m2 = np.zeros((P, 3), np.float32)
    g_con = np.zeros((P, 4), np.float32)
    g_op = np.zeros((P, 1), np.float32)
    g_col = np.zeros((P, C), np.float32)
    g_invd = np.zeros(P, np.float32) if dL_dinvdepth is not None else None
    pl = st["point_list"] if st["R"] > 0 else np.zeros(1, np.uint32)
    lib().gsro_set_backward_order(int(bool(reverse_order)))
    lib().gsro_render_backward(
        int(W), int(H), _p(st["ranges"], _u32), _p(pl, _u32), _p(_f32(bg), _f),
        _p(st["means2D"], _f), _p(st["conic_opacity"], _f), _p(_f32(colors), _f),
        _p(st["depths"], _f), _p(st["final_T"], _f), _p(st["n_contrib"], _u32),
        _p(_f32(dL_dcolor), _f), _p(_f32(dL_dinvdepth), _f), _mode(exact_exp),
        _p(g_m2, _f), _p(g_con, _f), _p(g_op, _f), _p(g_col, _f), _p(g_invd, _f))
    lib().gsro_set_backward_order(0)
    g_m3 = np.zeros((P, 3), np.float32)
    g_cov = np.zeros((P, 6), np.float32)
    g_sc = np.zeros((P, 3), np.float32)
    g_rot = np.zeros((P, 4), np.float32)
    cov3D = st["cov3D"] if cov3D_precomp is None else _f32(cov3D_precomp)
    lib().gsro_preprocess_backward(
        P, int(W), int(H), _p(means3D, _f), _p(st["radii"], _i), _p(_f32(scales), _f),
        float(scale_modifier), _p(_f32(rotations), _f), _p(_f32(opacities).reshape(-1), _f),
        _p(np.ascontiguousarray(cov3D, np.float32), _f), _p(_f32(view), _f), _p(_f32(proj), _f),
        float(tanx), float(tany), _p(g_m2, _f), _p(g_con, _f), _p(g_invd, _f),
        int(bool(antialiasing)), _p(g_op, _f), _p(g_m3, _f), _p(g_cov, _f), _p(g_sc, _f),
        _p(g_rot, _f))
    g_sh = np.zeros((P, 0, 3), np.float32)
    return g_m2, g_col, g_op, g_m3, g_cov, g_sh, g_sc, g_rot
