"""Per-frame avatar deformation on the GPU (C ABI include/gsr_deform.h, csrc/deform.hip).

Host-side mirror of the reference's deformation API, so GUAVA's callers keep their call shapes:

  lbs(betas, pose, v_template, shapedirs, posedirs, J_regressor, parents, lbs_weights,
      joints_offset=None, pose2rot=True, dtype)          -> (verts, J_transformed)
                                                         models/modules/flame/lbs.py:142-229
  lbs_wobeta(pose, v_shaped, posedirs, J_regressor, parents, lbs_weights, joints_offset=None,
             pose2rot=True, dtype)                       -> (verts, J_transformed, J, T, A)
                                                         lbs.py:255-333
  EHMDeformer(body, flame, ...).forward(body_param_dict, flame_param_dict)
                                                         -> EHM.forward's dict (modules/ehm/EHM.py:36-156)
  GaussianDeformer(vertex_gaussian_assets, uv_gaussian_assets, faces).forward(verts, T)
                                                         -> the deformed_assets dict of
                                                         Ubody_Gaussian.forward
                                                         (UbodyAvatar/ubody_gaussian.py:245-289)

Every call runs the gfx950 kernels on the current HIP stream of the inputs' device; there is no
CPU path (CPU tensors raise).  The k-major operand layouts the kernels want (shapedirs, lbs_weights
transposed) are made once per asset tensor and cached.
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib

_T_CACHE = {}


def _dev_check(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("guava_renderer_amd.deform runs on the GPU only (got a CPU tensor)")


def _f32(t):
    return t.detach().to(torch.float32).contiguous()


def _cached_t(t, fn):
    """fn(t) cached on the tensor's identity and version (asset tensors are static)."""
    key = (t.data_ptr(), tuple(t.shape), t._version, fn.__name__)
    hit = _T_CACHE.get(key)
    if hit is None:
        if len(_T_CACHE) > 16:
            _T_CACHE.clear()
        hit = fn(t)
        _T_CACHE[key] = hit
    return hit


def _shapedirs_t(sd):  # [V,3,NB] -> [NB, V*3]
    return _f32(sd).permute(2, 0, 1).reshape(sd.shape[2], -1).contiguous()


def _weights_t(w):  # [V,J] -> [J,V]
    return _f32(w).t().contiguous()


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _parents_host(parents):
    p = parents.detach().cpu().numpy() if torch.is_tensor(parents) else np.asarray(parents)
    return np.ascontiguousarray(p.astype(np.int32))


def _run_lbs(betas, pose, v_template, shapedirs, posedirs, J_regressor, parents, lbs_weights,
             joints_offset, pose2rot, want_all):
    _dev_check(pose, v_template, posedirs, J_regressor, lbs_weights, betas, shapedirs, joints_offset)
    dev = v_template.device
    B = pose.shape[0] if betas is None else max(betas.shape[0], pose.shape[0])
    Jn = J_regressor.shape[0]
    V = J_regressor.shape[1]
    if v_template.shape[-2:] != (V, 3):
        raise RuntimeError(f"v_template must be [.., {V}, 3], got {tuple(v_template.shape)}")
    if lbs_weights.shape != (V, Jn):
        raise RuntimeError(f"lbs_weights must be [{V}, {Jn}], got {tuple(lbs_weights.shape)}")
    vt = _f32(v_template)
    if vt.dim() == 3 and vt.shape[0] == 1 and B > 1:
        vt = vt[0]
    vt_stride = 0 if vt.dim() == 2 else V * 3
    if vt.dim() == 3 and vt.shape[0] != B:
        raise RuntimeError("v_template batch does not match the pose batch")
    pose = _f32(pose)
    if pose2rot:
        if pose.numel() != B * Jn * 3:
            raise RuntimeError(f"pose must hold B*J*3 = {B * Jn * 3} axis-angle values")
    elif pose.numel() != B * Jn * 9:
        raise RuntimeError(f"pose must hold B*J*9 = {B * Jn * 9} rotation-matrix values")
    NB = 0
    sd = None
    bt = None
    if betas is not None:
        NB = betas.shape[1]
        if shapedirs.shape != (V, 3, NB):
            raise RuntimeError(f"shapedirs must be [{V}, 3, {NB}], got {tuple(shapedirs.shape)}")
        sd = _cached_t(shapedirs, _shapedirs_t)
        bt = _f32(betas).expand(B, NB).contiguous()
    if Jn > 1 and posedirs.shape != (9 * (Jn - 1), 3 * V):
        raise RuntimeError(f"posedirs must be [{9 * (Jn - 1)}, {3 * V}], got {tuple(posedirs.shape)}")
    pd = _f32(posedirs)
    jreg = _f32(J_regressor)
    wt = _cached_t(lbs_weights, _weights_t)
    jo = _f32(joints_offset).expand(B, Jn, 3).contiguous() if joints_offset is not None else None
    par = _parents_host(parents)
    o = dict(dtype=torch.float32, device=dev)
    verts = torch.empty((B, V, 3), **o)
    jt = torch.empty((B, Jn, 3), **o)
    jr = torch.empty((B, Jn, 3), **o) if want_all else None
    T = torch.empty((B, V, 4, 4), **o) if want_all else None
    A = torch.empty((B, Jn, 4, 4), **o) if want_all else None
    L = _lib.load()
    ws = torch.empty((L.gsr_lbs_workspace_bytes(B, V, Jn, NB),), dtype=torch.uint8, device=dev)
    rc = L.gsr_lbs(B, V, Jn, NB, _ptr(vt), vt_stride, _ptr(bt), _ptr(sd), _ptr(pose),
                   1 if pose2rot else 0, _ptr(pd), _ptr(jreg),
                   par.ctypes.data_as(ctypes.c_void_p), _ptr(wt), _ptr(jo), _ptr(verts), _ptr(jt),
                   _ptr(jr), _ptr(T), _ptr(A), None, _ptr(ws), _stream(dev))
    _lib.check(rc, "gsr_lbs")
    return verts, jt, jr, T, A


def lbs(betas, pose, v_template, shapedirs, posedirs, J_regressor, parents, lbs_weights,
        joints_offset=None, pose2rot=True, dtype=torch.float32):
    """lbs.py:142-229 on the GPU: (verts [B,V,3], J_transformed [B,J,3])."""
    verts, jt, _, _, _ = _run_lbs(betas, pose, v_template, shapedirs, posedirs, J_regressor,
                                  parents, lbs_weights, joints_offset, pose2rot, False)
    return verts, jt


def lbs_wobeta(pose, v_shaped, posedirs, J_regressor, parents, lbs_weights, joints_offset=None,
               pose2rot=True, dtype=torch.float32):
    """lbs.py:255-333 on the GPU: (verts, J_transformed, J, T [B,V,4,4], A [B,J,4,4])."""
    return _run_lbs(None, pose, v_shaped, None, posedirs, J_regressor, parents, lbs_weights,
                    joints_offset, pose2rot, True)


def _seg(segs, dst, col, t, B, width=None):
    """Queue a gsr_pack_rows segment: columns [col, col + width) of dst [B, W] from t, a [B, ...] or
    [1, ...] tensor (one row per frame, or one row broadcast); t None leaves the columns to the zero
    fill."""
    if t is None:
        return
    t = _f32(t)
    rows = t.reshape(t.shape[0], -1) if t.dim() > 1 else t.reshape(1, -1)  # 1-D: one broadcast row
    if rows.shape[0] not in (1, B):
        raise RuntimeError(f"parameter batch {rows.shape[0]} does not match the frame batch {B}")
    w = rows.shape[1] if width is None else width
    if w > rows.shape[1] or col + w > dst.shape[1]:
        raise RuntimeError(f"parameter of width {rows.shape[1]} does not fit columns [{col}, {col + w}) "
                           f"of a {dst.shape[1]}-wide coefficient row")
    _dev_check(rows)
    segs.append((rows, dst, col, w, 0 if rows.shape[0] == 1 else rows.stride(0)))


def _fill_zeros(segs, dsts, B):
    """The segment table: every queued copy plus a zero segment for each column run no copy covers."""
    table = []
    for rows, dst, col, w, sstr in segs:
        if w > 0:
            table.append(_lib.RowSegment(rows.data_ptr(), dst.data_ptr() + 4 * col, sstr, dst.stride(0), w, 0))
    for dst in dsts:
        covered = sorted((col, col + w) for _, d, col, w, _ in segs if d is dst and w > 0)
        c = 0
        for a, e in covered + [(dst.shape[1], dst.shape[1])]:
            if a < c:
                raise RuntimeError("overlapping coefficient segments")
            if a > c:
                table.append(_lib.RowSegment(None, dst.data_ptr() + 4 * c, 0, dst.stride(0), a - c, 0))
            c = max(c, e)
    if len(table) > 16:
        raise RuntimeError("too many coefficient segments for one gsr_pack_rows launch")
    return table


class GaussianDeformer:
    """The Gaussian half of Ubody_Gaussian (ubody_gaussian.py:162-289) over precomputed LBS output.

    vertex_gaussian_assets: dict with 'rotations' [V,4] or [1,V,4] wxyz, 'scales', 'opacities',
    'colors' (the reference's vertex_gaussian_assets keys, :169-173); uv_gaussian_assets: 'rotations',
    'scales', 'opacities', 'local_pos', 'binding_face' [N], 'face_bary' [N,3], 'colors' (:175-185).
    The RGB sigmoid of :186-187 is applied once here, as the reference's constructor does."""

    def __init__(self, vertex_gaussian_assets, uv_gaussian_assets, faces, sh_degree=0,
                 apply_rgb_sigmoid=True):
        va, ua = vertex_gaussian_assets, uv_gaussian_assets

        def sq(t):
            t = t.detach()
            return _f32(t[0] if t.dim() == 3 and t.shape[0] == 1 else t)

        _dev_check(faces, va["rotations"], ua["rotations"])
        self.faces = faces.detach().to(torch.int32).contiguous()
        self.v_rot, self.v_scale = sq(va["rotations"]), sq(va["scales"])
        self.u_rot, self.u_scale = sq(ua["rotations"]), sq(ua["scales"])
        self.u_local = sq(ua["local_pos"])
        self.bind = ua["binding_face"].detach().reshape(-1).to(torch.int32).contiguous()
        self.bary = _f32(ua["face_bary"].detach().reshape(-1, 3))
        self.V, self.N = self.v_rot.shape[0], self.u_rot.shape[0]
        col = torch.cat([sq(va["colors"]), sq(ua["colors"])], 0)
        if apply_rgb_sigmoid:
            col[:, :3] = torch.sigmoid(col[:, :3])
        self.colors = col.contiguous()
        self.opacity = torch.cat([sq(va["opacities"]), sq(ua["opacities"])], 0).contiguous()
        self.sh_degree = sh_degree
        self.bad = torch.zeros(1, dtype=torch.int32, device=self.faces.device)

    def forward(self, verts, vert_transforms):
        """verts [B,V,3], vert_transforms [B,V,4,4] (EHM's vertices / ver_transform_mat) ->
        deformed_assets dict of Ubody_Gaussian.forward (ubody_gaussian.py:279-289)."""
        _dev_check(verts, vert_transforms)
        B, V = verts.shape[:2]
        if V != self.V:
            raise RuntimeError(f"expected {self.V} vertices, got {V}")
        P = self.V + self.N
        dev = verts.device
        # one allocation, three views; the rotations first (the kernel stores them as float4)
        buf = torch.empty((B * P * 10,), dtype=torch.float32, device=dev)
        rot = buf[:B * P * 4].view(B, P, 4)
        xyz = buf[B * P * 4:B * P * 7].view(B, P, 3)
        scl = buf[B * P * 7:].view(B, P, 3)
        if verts.dtype is not torch.float32 or not verts.is_contiguous():
            verts = _f32(verts)
        vt = vert_transforms
        if vt.dtype is not torch.float32 or not vt.is_contiguous():
            vt = _f32(vt)
        rc = _lib.load().gsr_deform_gaussians(
            B, V, self.faces.shape[0], self.N, _ptr(verts), _ptr(vt), _ptr(self.faces),
            _ptr(self.v_rot), 0, _ptr(self.v_scale), 0, _ptr(self.bind), _ptr(self.bary),
            _ptr(self.u_local), 0, _ptr(self.u_rot), 0, _ptr(self.u_scale), 0, _ptr(xyz), _ptr(rot),
            _ptr(scl), _ptr(self.bad), _stream(dev))
        _lib.check(rc, "gsr_deform_gaussians")
        return {"features_color": self.colors.expand(B, -1, -1), "xyz": xyz, "rotation": rot,
                "scaling": scl, "opacity": self.opacity.expand(B, -1, -1),
                "sh_degree": self.sh_degree, "smplx_xyz_deform": verts}

    __call__ = forward

    def bad_index(self):
        """True if any binding-face / face-vertex index was out of range (synchronises)."""
        return bool(self.bad.item())


def _host(x):
    return x.detach().cpu().numpy() if torch.is_tensor(x) else np.asarray(x)


def tile_base(base_kmajor, stream=None):
    """The 1-KB tiled layout of a k-major blend-shape base [K, M] on the device (gsr_lbs_tile_bases,
    include/gsr_deform.h GsrLbsSparse.*_tiled), for 16-byte loads in the blend kernels."""
    K, M = base_kmajor.shape
    L = _lib.load()
    out = torch.empty((int(L.gsr_lbs_tiled_floats(K, M)),), dtype=torch.float32, device=base_kmajor.device)
    b = base_kmajor.contiguous()
    _lib.check(L.gsr_lbs_tile_bases(K, M, b.data_ptr(), out.data_ptr(), stream or _stream(base_kmajor.device)),
               "gsr_lbs_tile_bases")
    return out


def sparse_lbs_assets(J_regressor, lbs_weights, device):
    """GsrLbsSparse (include/gsr_deform.h) of one model's dense assets, built once on the host: the
    J_regressor's nonzeros as CSR rows (vertex order) and, when every vertex has at most 16 nonzero
    skinning weights, the weights as [K, V] (joint, weight) pairs in joint order (weight-0 padding).
    Returns (struct, tensors kept alive by the caller)."""
    jr = np.ascontiguousarray(_host(J_regressor), dtype=np.float32)
    w = np.ascontiguousarray(_host(lbs_weights), dtype=np.float32)
    J, V = jr.shape
    nz = jr != 0
    row = np.concatenate([[0], np.cumsum(nz.sum(1))]).astype(np.int32)
    col = np.nonzero(nz)[1].astype(np.int32)  # row-major: vertex order inside each row
    val = jr[nz].astype(np.float32)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=device)  # noqa: E731
    keep = [t(row), t(col if col.size else np.zeros(1, np.int32)), t(val if val.size else np.zeros(1, np.float32))]
    sp = _lib.LbsSparse(keep[0].data_ptr(), keep[1].data_ptr(), keep[2].data_ptr(), 0, 0, None, None)
    wnz = w != 0
    K = int(wnz.sum(1).max()) if V else 0
    if 1 <= K <= 16:
        order = np.argsort(~wnz, axis=1, kind="stable")[:, :K]  # each vertex's nonzero joints, in order
        sj = np.where(np.take_along_axis(wnz, order, 1), order, 0).astype(np.int32)
        sw = np.where(np.take_along_axis(wnz, order, 1), np.take_along_axis(w, sj, 1), 0.0)
        keep += [t(sj.T), t(sw.T.astype(np.float32))]
        sp.skin_k = K
        sp.skin_joint = keep[3].data_ptr()
        sp.skin_weight = keep[4].data_ptr()
    return sp, keep


class EHMDeformer:
    """EHM.forward (models/modules/ehm/EHM.py:36-156) for B frames on the GPU: FLAME head lbs ->
    eyelids and head scale -> body blend shapes and joints -> head splice -> body lbs_wobeta, with
    every per-frame step a gfx950 kernel (gsr_pack_rows, gsr_lbs, gsr_blend_joints, gsr_splice_head)
    and no host synchronisation or torch glue launches.

    body / flame: dicts of the LBS assets in the reference layouts (v_template [V,3], shapedirs
    [V,3,NB], posedirs, J_regressor, parents, lbs_weights); smplx2flame_ind [Nh] (SMPLX.py:191);
    l_eyelid / r_eyelid [Nh,3] (FLAME.py:105-106).  The k-major copies are made once here.
    Inputs of forward() are the reference's parameter dicts (tensors on the device)."""

    HEAD_REF = (3, 5)    # head_joints[:, 3:5] (EHM.py:123)
    BODY_REF = (23, 25)  # tbody_joints[:, 23:25]

    def __init__(self, body, flame, smplx2flame_ind, l_eyelid, r_eyelid, device="cuda"):
        dev = torch.device(device)
        t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)  # noqa: E731
        self.dev = dev
        self.body = {k: (t(v) if k != "parents" else np.asarray(v, np.int32)) for k, v in body.items()}
        self.flame = {k: (t(v) if k != "parents" else np.asarray(v, np.int32)) for k, v in flame.items()}
        for a in (self.body, self.flame):
            a["shapedirs_t"] = _shapedirs_t(a["shapedirs"])
            a["lbs_weights_t"] = _weights_t(a["lbs_weights"])
        # the sparse J_regressor / skinning weights (GSR_LBS_SPARSE=0: the dense kernels, A/B)
        self.sparse = {}
        if os.environ.get("GSR_LBS_SPARSE", "1") != "0":
            for name, a in (("body", body), ("flame", flame)):
                self.sparse[name] = sparse_lbs_assets(a["J_regressor"], a["lbs_weights"], dev)
        # the blend-shape bases as 16-byte tiles (GSR_BLEND_TILED=0 in the library: the k-major kernels)
        for name, a in (("body", self.body), ("flame", self.flame)):
            if name in self.sparse:
                sp, keep = self.sparse[name]
                bases = (a["shapedirs_t"], _f32(a["posedirs"]))
                tl = [tile_base(x) if x.numel() else None for x in bases]
                keep += tl
                sp.shapedirs_tiled, sp.posedirs_tiled = (x.data_ptr() if x is not None else None for x in tl)
                # the K x M each base was tiled for (the library refuses calls of another shape)
                (sp.shapedirs_tiled_k, sp.shapedirs_tiled_m), (sp.posedirs_tiled_k, sp.posedirs_tiled_m) = (
                    tuple(x.shape) if x.numel() else (0, 0) for x in bases)
        self.head_index = t(np.asarray(smplx2flame_ind, np.int32))
        self.l_eyelid, self.r_eyelid = t(np.asarray(l_eyelid, np.float32)), t(np.asarray(r_eyelid, np.float32))
        self.bad = torch.zeros(1, dtype=torch.int32, device=dev)
        self._ws = {}
        self._ehm = self._ehm_struct()
        self._ehm_ref = ctypes.byref(self._ehm)
        # GSR_EHM_ONECALL=0: the per-step C calls from Python (forward_calls), A/B
        self.one_call = os.environ.get("GSR_EHM_ONECALL", "1") != "0"

    def _ehm_struct(self):
        """GsrEhm (include/gsr_deform.h) of this avatar, made once; the objects it points to are
        attributes of self."""
        def model(a, name):
            m = _lib.EhmModel()
            m.J, m.V = a["J_regressor"].shape
            m.NB = a["shapedirs"].shape[2]
            m.v_template, m.shapedirs_t = a["v_template"].data_ptr(), a["shapedirs_t"].data_ptr()
            a["posedirs"] = _f32(a["posedirs"])
            m.posedirs, m.J_regressor = a["posedirs"].data_ptr(), a["J_regressor"].data_ptr()
            m.lbs_weights_t = a["lbs_weights_t"].data_ptr()
            a["parents"] = np.ascontiguousarray(a["parents"], np.int32)
            m.parents_host = a["parents"].ctypes.data
            if name in self.sparse:
                m.sparse = ctypes.pointer(self.sparse[name][0])
            return m
        for a in (self.body, self.flame):
            for k in ("v_template", "J_regressor"):
                a[k] = _f32(a[k])
        e = _lib.Ehm()
        e.flame, e.body = model(self.flame, "flame"), model(self.body, "body")
        e.head_index, e.l_eyelid, e.r_eyelid = (x.data_ptr() for x in (self.head_index, self.l_eyelid, self.r_eyelid))
        e.N_head = self.head_index.shape[0]
        e.hj0, e.hj1 = self.HEAD_REF
        e.bj0, e.bj1 = self.BODY_REF
        e.bad_index_flag = self.bad.data_ptr()
        return e

    def _workspace(self, B, V, J, NB):
        # one per stream: batches in flight on different streams must not share scratch
        key = (B, V, J, NB, torch.cuda.current_stream(self.dev).cuda_stream)
        if key not in self._ws:
            n = _lib.load().gsr_lbs_workspace_bytes(B, V, J, NB)
            self._ws[key] = torch.empty((n,), dtype=torch.uint8, device=self.dev)
        return self._ws[key]

    def forward(self, body_param_dict, flame_param_dict):
        """EHM.forward through gsr_ehm_forward: the parameter descriptors and one C call."""
        if not self.one_call:
            return self.forward_calls(body_param_dict, flame_param_dict)
        bp, fp = body_param_dict, flame_param_dict
        if bp.get("hand_scale") is not None:
            raise NotImplementedError("hand_scale (EHM.py:126-132) needs the MANO vertex map, not bundled")
        B = fp["shape_params"].shape[0]
        prm = (_lib.EhmParam * 13)()
        keep = []
        for i, t in enumerate((fp["shape_params"], fp["expression_params"], fp.get("jaw_params"),
                               fp.get("eye_pose_params"), fp.get("eyelid_params"), bp["shape"], bp["exp"],
                               bp.get("global_pose"), bp.get("body_pose"), bp["left_hand_pose"],
                               bp["right_hand_pose"], bp.get("head_scale"), bp.get("joints_offset"))):
            if t is None:
                continue
            if t.dtype is not torch.float32 or not t.is_contiguous():
                t = _f32(t)
                keep.append(t)
            if not t.is_cuda:
                raise RuntimeError("guava_renderer_amd.deform runs on the GPU only (got a CPU tensor)")
            rows = t.shape[0] if t.dim() > 1 else 1  # 1-D: one row for every frame
            if rows != 1 and rows != B:
                raise RuntimeError(f"parameter batch {rows} does not match the frame batch {B}")
            q = prm[i]
            q.p = t.data_ptr()
            q.width = t.numel() // rows if rows else 0
            q.row_stride = q.width if rows > 1 else 0
        Vb, Jb = self._ehm.body.V, self._ehm.body.J
        n3, n16 = B * Vb * 3, B * Vb * 16
        j3, j16 = B * Jb * 3, B * Jb * 16
        # one allocation for the five outputs; the 4x4 transforms first (stored as float4)
        buf = torch.empty((n16 + j16 + n3 + 2 * j3,), dtype=torch.float32, device=self.dev)
        T = buf[:n16].view(B, Vb, 4, 4)
        A = buf[n16:n16 + j16].view(B, Jb, 4, 4)
        o = n16 + j16
        verts, J, jt2 = buf[o:o + n3].view(B, Vb, 3), buf[o + n3:o + n3 + j3].view(B, Jb, 3), buf[o + n3 + j3:].view(B, Jb, 3)
        out = _lib.EhmOutputs(verts.data_ptr(), J.data_ptr(), jt2.data_ptr(), T.data_ptr(), A.data_ptr())
        st = torch.cuda.current_stream(self.dev).cuda_stream
        ws = self._ws.get((B, st))
        if ws is None:
            n = _lib.load().gsr_ehm_workspace_bytes(self._ehm_ref, B)
            ws = self._ws[(B, st)] = torch.empty((n,), dtype=torch.uint8, device=self.dev)
        _lib.check(_lib.load().gsr_ehm_forward(self._ehm_ref, B, prm, ctypes.byref(out), ws.data_ptr(), st),
                   "gsr_ehm_forward")
        return {"vertices": verts, "joints": J, "joints_transform": jt2, "ver_transform_mat": T,
                "joint_transform_mat": A}

    def forward_calls(self, body_param_dict, flame_param_dict):
        """EHM.forward as Python-issued C calls per step (gsr_pack_rows, gsr_lbs_sp, gsr_blend_joints_sp,
        gsr_splice_head, gsr_lbs_sp): the same kernels and results as forward()."""
        L = _lib.load()
        st = _stream(self.dev)
        bp, fp = body_param_dict, flame_param_dict
        if bp.get("hand_scale") is not None:
            raise NotImplementedError("hand_scale (EHM.py:126-132) needs the MANO vertex map, not bundled")
        fa, ba = self.flame, self.body
        B = fp["shape_params"].shape[0]
        o = dict(dtype=torch.float32, device=self.dev)
        Vh, Jh, NBh = fa["J_regressor"].shape[1], fa["J_regressor"].shape[0], fa["shapedirs"].shape[2]
        Vb, Jb, NBb = ba["J_regressor"].shape[1], ba["J_regressor"].shape[0], ba["shapedirs"].shape[2]
        # the coefficient rows of both LBS calls, assembled by ONE gsr_pack_rows launch (the
        # reference's torch.cat / zeros / expand glue): FLAME betas = shape ++ expression ++ 0 and
        # pose = 0 global, 0 neck, jaw, eyes (EHM.py:41-48); SMPL-X shape (cut or zero-padded to
        # n_shape) ++ exp (:101-106); body pose = global, body, 0 jaw, 0 eyes, hands (:94-112)
        hs = bp.get("head_scale")
        widths = (NBh, 3 * Jh, NBb, 3 * Jb, 3 if hs is not None else 0)
        buf = torch.empty((sum(widths) * B,), **o)
        views, off = [], 0
        for w in widths:
            views.append(buf[off:off + B * w].view(B, w))
            off += B * w
        betas_h, pose_h, sc, pose, hsb = views
        segs = []
        # FLAME betas: shape zero-padded to flame.n_shape, then the expression (EHM.py:53-62)
        n_shape_h = NBh - fp["expression_params"].shape[-1]
        if fp["shape_params"].shape[-1] > n_shape_h:
            raise ValueError(f"FLAME shape_params ({fp['shape_params'].shape[-1]}) + expression_params "
                             f"({fp['expression_params'].shape[-1]}) wider than the FLAME blend ({NBh})")
        _seg(segs, betas_h, 0, fp["shape_params"], B)
        _seg(segs, betas_h, n_shape_h, fp["expression_params"], B)
        _seg(segs, pose_h, 6, fp["jaw_params"], B)
        _seg(segs, pose_h, 9, fp["eye_pose_params"], B)
        n_shape = NBb - bp["exp"].shape[-1]
        _seg(segs, sc, 0, bp["shape"], B, width=min(n_shape, bp["shape"].shape[-1]))
        _seg(segs, sc, n_shape, bp["exp"], B)
        for name, wd in (("global_pose", 3), ("body_pose", 63)):  # (EHM.py:107-114: no prefix is taken)
            t_ = bp.get(name)
            if t_ is not None and t_.numel() // max(1, t_.shape[0] if t_.dim() > 1 else 1) != wd:
                raise ValueError(f"{name} must be {wd} columns wide")
        _seg(segs, pose, 0, bp.get("global_pose"), B, width=3)
        _seg(segs, pose, 3, bp.get("body_pose"), B, width=63)
        _seg(segs, pose, 75, bp["left_hand_pose"], B)
        _seg(segs, pose, 120, bp["right_hand_pose"], B)
        if hs is not None:
            _seg(segs, hsb, 0, hs, B)
        table = _fill_zeros(segs, views, B)
        _lib.check(L.gsr_pack_rows(B, len(table), (_lib.RowSegment * len(table))(*table), st), "gsr_pack_rows")
        # FLAME head (EHM.py:41-75)
        hv = torch.empty((B, Vh, 3), **o)
        hj = torch.empty((B, Jh, 3), **o)
        sph = ctypes.byref(self.sparse["flame"][0]) if "flame" in self.sparse else None
        spb = ctypes.byref(self.sparse["body"][0]) if "body" in self.sparse else None
        rc = L.gsr_lbs_sp(B, Vh, Jh, NBh, _ptr(fa["v_template"]), 0, _ptr(betas_h),
                          _ptr(fa["shapedirs_t"]), _ptr(pose_h), 1, _ptr(fa["posedirs"]),
                          _ptr(fa["J_regressor"]), fa["parents"].ctypes.data_as(ctypes.c_void_p),
                          _ptr(fa["lbs_weights_t"]), None, _ptr(hv), _ptr(hj), None, None, None, None,
                          _ptr(self._workspace(B, Vh, Jh, NBh)), sph, st)
        _lib.check(rc, "gsr_lbs (FLAME head)")
        # body template (EHM.py:101-118): blend shapes of shape ++ exp, regressed joints + offset
        joff = _f32(bp["joints_offset"]) if bp.get("joints_offset") is not None else None
        vt = torch.empty((B, Vb, 3), **o)
        tj = torch.empty((B, Jb, 3), **o)
        _lib.check(L.gsr_blend_joints_sp(B, Vb, Jb, NBb, _ptr(ba["v_template"]), 0, _ptr(sc),
                                         _ptr(ba["shapedirs_t"]), _ptr(ba["J_regressor"]), _ptr(joff),
                                         _ptr(vt), _ptr(tj), spb, st), "gsr_blend_joints")
        # head splice (EHM.py:72-75, 121-124)
        eyelid = _f32(fp["eyelid_params"]) if fp.get("eyelid_params") is not None else None
        _lib.check(L.gsr_splice_head(B, Vb, Vh, _ptr(self.head_index), _ptr(hv), _ptr(self.r_eyelid),
                                     _ptr(self.l_eyelid), _ptr(eyelid), _ptr(hsb) if hs is not None else None, _ptr(hj), Jh,
                                     self.HEAD_REF[0], self.HEAD_REF[1], _ptr(tj), Jb, self.BODY_REF[0],
                                     self.BODY_REF[1], _ptr(vt), _ptr(self.bad), st), "gsr_splice_head")
        verts = torch.empty((B, Vb, 3), **o)
        jt2 = torch.empty((B, Jb, 3), **o)
        J = torch.empty((B, Jb, 3), **o)
        T = torch.empty((B, Vb, 4, 4), **o)
        A = torch.empty((B, Jb, 4, 4), **o)
        rc = L.gsr_lbs_sp(B, Vb, Jb, 0, _ptr(vt), Vb * 3, None, None, _ptr(pose), 1, _ptr(ba["posedirs"]),
                          _ptr(ba["J_regressor"]), ba["parents"].ctypes.data_as(ctypes.c_void_p),
                          _ptr(ba["lbs_weights_t"]), _ptr(joff), _ptr(verts), _ptr(jt2), _ptr(J), _ptr(T),
                          _ptr(A), None, _ptr(self._workspace(B, Vb, Jb, 0)), spb, st)
        _lib.check(rc, "gsr_lbs (SMPL-X body)")
        return {"vertices": verts, "joints": J, "joints_transform": jt2, "ver_transform_mat": T,
                "joint_transform_mat": A}

    __call__ = forward
