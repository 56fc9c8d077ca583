"""Independent float64 dense restatement of the rasterizer in torch (test infrastructure).

Written from the reference's math (forward.cu:74-397, auxiliary.h:40-176) in glm's matrix
conventions, vectorised over pixels, with autograd providing the backward.  It shares no code with
the C oracle; it is used to pin the oracle (forward within float32 rounding, gradients within 1e-3
relative) because the reference ships no tests or golden vectors for this path.

Reference quirks reproduced so that autograd equals the reference's hand-written backward:
  * alpha = min(0.99, o*G) with the gradient of o*G (backward.cu:619, 635 ignore the clamp);
  * the EWA clamp of t.xy zeroes the gradient outside the limits (backward.cu:182-183);
  * dL/dmeans2D is the gradient w.r.t. the NDC position (ddelx_dx = W/2, backward.cu:527);
  * tile membership (the discrete rect test) is taken as given.
"""
import torch

C = 32


def _glm(*a):
    """glm::mat3(a0..a8) -> tensor [..., col, row]."""
    cols = [torch.stack(a[3 * c:3 * c + 3], -1) for c in range(3)]
    return torch.stack(cols, -2)


def _mul(A, B):
    # glm: Result[c][r] = sum_k A[k][r] * B[c][k]
    return torch.einsum("...kr,...ck->...cr", A, B)


def _tr(A):
    return A.transpose(-1, -2)


def project(means3D, scales, rotations, view, proj, W, H, tanx, tany, scale_mod=1.0, ndc_offset=None):
    """Per-Gaussian projection. Returns dict of tensors (float64)."""
    V = view.reshape(4, 4)
    Pm = proj.reshape(4, 4)
    p = means3D
    pv = p @ V[:3, :3] + V[3, :3]
    ph = p @ Pm[:3, :] + Pm[3, :]
    pw = 1.0 / (ph[:, 3] + 1e-7)
    ndc = ph[:, :2] * pw[:, None]
    if ndc_offset is not None:
        ndc = ndc + ndc_offset[:, :2]
    # cov3D (forward.cu:114-148)
    s = scale_mod * scales
    z0 = torch.zeros_like(s[:, 0])
    o1 = torch.ones_like(s[:, 0])
    S = _glm(s[:, 0], z0, z0, z0, s[:, 1], z0, z0, z0, s[:, 2])
    r, x, y, zq = rotations[:, 0], rotations[:, 1], rotations[:, 2], rotations[:, 3]
    R = _glm(1 - 2 * (y * y + zq * zq), 2 * (x * y - r * zq), 2 * (x * zq + r * y),
             2 * (x * y + r * zq), 1 - 2 * (x * x + zq * zq), 2 * (y * zq - r * x),
             2 * (x * zq - r * y), 2 * (y * zq + r * x), 1 - 2 * (x * x + y * y))
    M = _mul(S, R)
    Sig = _mul(_tr(M), M)
    # cov2D (forward.cu:74-109)
    fx = W / (2.0 * tanx)
    fy = H / (2.0 * tany)
    t = pv
    limx, limy = 1.3 * tanx, 1.3 * tany
    tx = torch.clamp(t[:, 0] / t[:, 2], -limx, limx) * t[:, 2]
    ty = torch.clamp(t[:, 1] / t[:, 2], -limy, limy) * t[:, 2]
    tz = t[:, 2]
    J = _glm(fx / tz, z0, -(fx * tx) / (tz * tz), z0, fy / tz, -(fy * ty) / (tz * tz), z0, z0, z0)
    Wm = _glm(*[V.reshape(-1)[k].expand_as(z0) for k in (0, 4, 8, 1, 5, 9, 2, 6, 10)])
    T = _mul(Wm, J)
    cov = _mul(_mul(_tr(T), _tr(Sig)), T)
    cxx = cov[:, 0, 0] + 0.3
    cxy = cov[:, 0, 1]
    cyy = cov[:, 1, 1] + 0.3
    det = cxx * cyy - cxy * cxy
    conic = torch.stack([cyy / det, -cxy / det, cxx / det], -1)
    pix = ((ndc + 1.0) * torch.tensor([W, H], dtype=ndc.dtype) - 1.0) * 0.5
    return dict(depth=tz, means2D=pix, conic=conic, cov3D=Sig, o1=o1)


def render(proj_out, opacities, colors, bg, W, H, tile_lists, exact_exp=None):
    """Front-to-back blend over each tile's given depth-sorted list (forward.cu:274-397).
    tile_lists: dict tile -> array of Gaussian indices (sorted).  Returns (color[C,H,W],
    invdepth[H,W], final_T[H,W], n_contrib[H,W])."""
    gx = (W + 15) // 16
    dt = proj_out["means2D"].dtype
    out = torch.zeros((C, H, W), dtype=dt)
    inv_img = torch.zeros((H, W), dtype=dt)
    T_img = torch.ones((H, W), dtype=dt)
    nc_img = torch.zeros((H, W), dtype=torch.int64)
    out = out + bg.reshape(C, 1, 1) * 0  # keep dtype/graph
    rows = []
    for tile, lst in tile_lists.items():
        tx, ty = tile % gx, tile // gx
        ys = torch.arange(ty * 16, min(ty * 16 + 16, H))
        xs = torch.arange(tx * 16, min(tx * 16 + 16, W))
        if len(ys) == 0 or len(xs) == 0:
            continue
        YY, XX = torch.meshgrid(ys, xs, indexing="ij")
        pfx = XX.reshape(-1).to(dt)
        pfy = YY.reshape(-1).to(dt)
        npx = pfx.shape[0]
        Tt = torch.ones(npx, dtype=dt)
        Cc = torch.zeros((npx, C), dtype=dt)
        inv = torch.zeros(npx, dtype=dt)
        done = torch.zeros(npx, dtype=torch.bool)
        last = torch.zeros(npx, dtype=torch.int64)
        for pos, g in enumerate(lst):
            g = int(g)
            m = proj_out["means2D"][g]
            co = proj_out["conic"][g]
            dx = m[0] - pfx
            dy = m[1] - pfy
            power = -0.5 * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy
            G = torch.exp(power)
            oG = opacities[g] * G
            alpha = oG - torch.relu(oG - 0.99).detach()
            take = (~done) & ~(power > 0) & ~(alpha < 1.0 / 255.0)
            test_T = Tt * (1 - alpha)
            term = take & (test_T < 1e-4)
            contrib = take & ~term
            w = torch.where(contrib, alpha * Tt, torch.zeros_like(alpha))
            Cc = Cc + w[:, None] * colors[g][None, :]
            inv = inv + w / proj_out["depth"][g]
            Tt = torch.where(contrib, test_T, Tt)
            last = torch.where(contrib, torch.full_like(last, pos + 1), last)
            done = done | term
        rows.append((YY.reshape(-1), XX.reshape(-1), Cc, inv, Tt, last))
    # assemble (functional, to keep autograd)
    flat_C = torch.zeros((H * W, C), dtype=dt)
    flat_inv = torch.zeros(H * W, dtype=dt)
    flat_T = torch.ones(H * W, dtype=dt)
    for YY, XX, Cc, inv, Tt, last in rows:
        idx = YY * W + XX
        flat_C = flat_C.index_put((idx,), Cc)
        flat_inv = flat_inv.index_put((idx,), inv)
        flat_T = flat_T.index_put((idx,), Tt)
        nc_img.view(-1)[idx] = last
    out = (flat_C + flat_T[:, None] * bg[None, :]).T.reshape(C, H, W)
    return out, flat_inv.reshape(H, W), flat_T.reshape(H, W), nc_img
