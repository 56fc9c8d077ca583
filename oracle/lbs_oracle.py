"""CPU oracle of the per-frame avatar deformation (numpy, float64 arithmetic).

TEST INFRASTRUCTURE ONLY: imported by tests/ (and __graft_entry__.smoke()) as the checker of the
gfx950 deform path (guava_renderer_amd/csrc/deform.hip); the product never imports it.

A restatement of the reference's algorithm, each function citing what it follows
(/root/reference/...):
  batch_rodrigues        models/modules/flame/lbs.py:379-410
  blend_shapes           lbs.py:355-376
  vertices2joints        lbs.py:335-352
  batch_rigid_transform  lbs.py:426-482 (transform_mat :413-423)
  lbs                    lbs.py:142-229
  lbs_wobeta             lbs.py:255-333
  face_orientation       utils/graphics_utils.py:52-80 (compute_face_orientation, return_scale)
  rotmat_to_unitquat     roma 1.5.3 (requirements.txt:6; not vendored, not installed here): the
                         published scipy-derived decision scheme (Rotation.from_matrix), xyzw
  quat_product           roma 1.5.3 quat_product, xyzw Hamilton product
  deform_gaussians       models/UbodyAvatar/ubody_gaussian.py:252-278
Pinning: lbs / lbs_wobeta / batch_rodrigues / batch_rigid_transform against outputs of the
reference's own lbs.py run in the build container (tests/golden/lbs_golden.npz,
tests/golden/make_lbs_golden.py); the roma and graphics_utils restatements (not importable here:
roma absent, graphics_utils needs pytorch3d/lightning) are "parity unpinned" against the reference
and checked by properties (unit norm, rotation round trip through an independent quaternion->matrix
formula and scipy's Rotation.from_matrix, Hamilton composition, right-handed orthonormal frames).
  ehm_forward            models/modules/ehm/EHM.py:36-137 (composition of the above + head splice)
"""
import numpy as np


def batch_rodrigues(rot_vecs):
    """[N,3] axis-angle -> [N,3,3] (lbs.py:394-410: angle = |r + 1e-8|, dir = r / angle)."""
    r = np.asarray(rot_vecs, np.float64).reshape(-1, 3)
    angle = np.linalg.norm(r + 1e-8, axis=1, keepdims=True)
    d = r / angle
    c = np.cos(angle)[:, :, None]
    s = np.sin(angle)[:, :, None]
    z = np.zeros(r.shape[0])
    K = np.stack([z, -d[:, 2], d[:, 1], d[:, 2], z, -d[:, 0], -d[:, 1], d[:, 0], z], 1).reshape(-1, 3, 3)
    return np.eye(3)[None] + s * K + (1 - c) * (K @ K)


def blend_shapes(betas, shapedirs):
    """einsum('bl,mkl->bmk') (lbs.py:375)."""
    return np.einsum("bl,mkl->bmk", np.asarray(betas, np.float64), np.asarray(shapedirs, np.float64))


def vertices2joints(J_regressor, vertices):
    """einsum('bik,ji->bjk') (lbs.py:352)."""
    return np.einsum("bik,ji->bjk", np.asarray(vertices, np.float64), np.asarray(J_regressor, np.float64))


def batch_rigid_transform(rot_mats, joints, parents):
    """(posed_joints [B,J,3], rel_transforms A [B,J,4,4]) (lbs.py:450-483)."""
    rot_mats = np.asarray(rot_mats, np.float64)
    joints = np.asarray(joints, np.float64)
    B, J = joints.shape[:2]
    rel = joints.copy()
    rel[:, 1:] -= joints[:, parents[1:]]
    tm = np.zeros((B, J, 4, 4))
    tm[:, :, :3, :3] = rot_mats
    tm[:, :, :3, 3] = rel
    tm[:, :, 3, 3] = 1.0
    chain = [tm[:, 0]]
    for i in range(1, J):
        chain.append(chain[parents[i]] @ tm[:, i])
    T = np.stack(chain, 1)
    posed = T[:, :, :3, 3].copy()
    jh = np.concatenate([joints, np.zeros((B, J, 1))], -1)[..., None]  # F.pad(joints, [0,0,0,1])
    A = T.copy()
    A[:, :, :, 3] -= (T @ jh)[..., 0]
    return posed, A


def _skin(v_posed, lbs_weights, A):
    B, J = A.shape[:2]
    T = np.einsum("vj,bjk->bvk", np.asarray(lbs_weights, np.float64), A.reshape(B, J, 16)).reshape(B, -1, 4, 4)
    vh = np.concatenate([v_posed, np.ones(v_posed.shape[:2] + (1,))], -1)
    verts = np.einsum("bvij,bvj->bvi", T, vh)[..., :3]
    return verts, T


def _pose_rot(pose, B, pose2rot):
    if pose2rot:
        return batch_rodrigues(np.asarray(pose).reshape(-1, 3)).reshape(B, -1, 3, 3)
    return np.asarray(pose, np.float64).reshape(B, -1, 3, 3)


def lbs_wobeta(pose, v_shaped, posedirs, J_regressor, parents, lbs_weights, joints_offset=None,
               pose2rot=True):
    """(verts, J_transformed, J, T [B,V,4,4], A [B,J,4,4]) as lbs.py:255-333."""
    v_shaped = np.asarray(v_shaped, np.float64)
    B = np.asarray(pose).shape[0]
    if v_shaped.shape[0] != B:
        v_shaped = np.broadcast_to(v_shaped, (B,) + v_shaped.shape[1:])
    J = vertices2joints(J_regressor, v_shaped)
    if joints_offset is not None:
        J = J + np.asarray(joints_offset, np.float64)
    rot = _pose_rot(pose, B, pose2rot)
    feat = (rot[:, 1:] - np.eye(3)).reshape(B, -1)
    v_posed = (feat @ np.asarray(posedirs, np.float64)).reshape(B, -1, 3) + v_shaped
    Jt, A = batch_rigid_transform(rot, J, np.asarray(parents))
    verts, T = _skin(v_posed, lbs_weights, A)
    return verts, Jt, J, T, A


def lbs(betas, pose, v_template, shapedirs, posedirs, J_regressor, parents, lbs_weights,
        joints_offset=None, pose2rot=True):
    """(verts, J_transformed) as lbs.py:142-229; also returns (T, A, J) for checking."""
    v_shaped = np.asarray(v_template, np.float64) + blend_shapes(betas, shapedirs)
    verts, Jt, J, T, A = lbs_wobeta(pose, v_shaped, posedirs, J_regressor, parents, lbs_weights,
                                    joints_offset, pose2rot)
    return verts, Jt, J, T, A, v_shaped


def rotmat_to_unitquat(R):
    """roma.rotmat_to_unitquat: [...,3,3] -> ([...,4] xyzw, decision margin [...]).  The margin is
    the gap between the chosen and the runner-up decision value: where it is tiny, a float32
    evaluation may legitimately take the other branch."""
    m = np.asarray(R, np.float64).reshape(-1, 3, 3)
    n = m.shape[0]
    dec = np.empty((n, 4))
    dec[:, :3] = np.diagonal(m, axis1=1, axis2=2)
    dec[:, 3] = dec[:, :3].sum(1)
    ch = dec.argmax(1)
    srt = np.sort(dec, 1)
    margin = srt[:, 3] - srt[:, 2]
    q = np.empty((n, 4))
    ind = np.nonzero(ch != 3)[0]
    i = ch[ind]
    j = (i + 1) % 3
    k = (j + 1) % 3
    q[ind, i] = 1 - dec[ind, 3] + 2 * m[ind, i, i]
    q[ind, j] = m[ind, j, i] + m[ind, i, j]
    q[ind, k] = m[ind, k, i] + m[ind, i, k]
    q[ind, 3] = m[ind, k, j] - m[ind, j, k]
    ind = np.nonzero(ch == 3)[0]
    q[ind, 0] = m[ind, 2, 1] - m[ind, 1, 2]
    q[ind, 1] = m[ind, 0, 2] - m[ind, 2, 0]
    q[ind, 2] = m[ind, 1, 0] - m[ind, 0, 1]
    q[ind, 3] = 1 + dec[ind, 3]
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    shp = np.asarray(R).shape[:-2]
    return q.reshape(shp + (4,)), margin.reshape(shp)


def quat_product(p, q):
    """roma.quat_product (xyzw)."""
    p = np.asarray(p, np.float64)
    q = np.asarray(q, np.float64)
    v = p[..., 3:] * q[..., :3] + q[..., 3:] * p[..., :3] + np.cross(p[..., :3], q[..., :3])
    w = p[..., 3] * q[..., 3] - (p[..., :3] * q[..., :3]).sum(-1)
    return np.concatenate([v, w[..., None]], -1)


def wxyz_to_xyzw(q):
    return np.concatenate([q[..., 1:], q[..., :1]], -1)


def xyzw_to_wxyz(q):
    return np.concatenate([q[..., 3:], q[..., :3]], -1)


def face_orientation(verts, faces):
    """compute_face_orientation(verts, faces, return_scale=True) (graphics_utils.py:61-80):
    ([...,F,3,3] columns a0 a1 a2, [...,F,1] scale)."""
    v = np.asarray(verts, np.float64)
    f = np.asarray(faces).astype(np.int64)
    v0, v1, v2 = v[..., f[:, 0], :], v[..., f[:, 1], :], v[..., f[:, 2], :]

    def length(x):
        return np.sqrt(np.maximum((x * x).sum(-1, keepdims=True), 1e-20))

    a0 = (v1 - v0) / length(v1 - v0)
    c1 = np.cross(a0, v2 - v0)
    a1 = c1 / length(c1)
    c2 = np.cross(a1, a0)
    a2 = -(c2 / length(c2))
    orient = np.stack([a0, a1, a2], -1)
    scale = (length(v1 - v0) + np.abs((a2 * (v2 - v0)).sum(-1, keepdims=True))) / 2
    return orient, scale


def deform_gaussians(verts, vert_transforms, faces, vtx_rotations, vtx_scales, binding_face,
                     face_bary, local_xyz, uv_rotations, uv_scales):
    """Ubody_Gaussian.forward's Gaussian assembly (ubody_gaussian.py:252-278) for B frames.
    verts [B,V,3], vert_transforms [B,V,4,4]; canonical assets [n,k] or [B,n,k].
    Returns dict(xyz [B,P,3], rotation [B,P,4] wxyz, scaling [B,P,3], margin [B,P])."""
    verts = np.asarray(verts, np.float64)
    B, V = verts.shape[:2]

    def per_frame(x):
        x = np.asarray(x, np.float64)
        return np.broadcast_to(x, (B,) + x.shape) if x.ndim == 2 else x

    qd, m_v = rotmat_to_unitquat(np.asarray(vert_transforms, np.float64)[:, :, :3, :3])
    qv = quat_product(qd, wxyz_to_xyzw(per_frame(vtx_rotations)))
    qv = xyzw_to_wxyz(qv)
    qv = qv / np.maximum(np.linalg.norm(qv, axis=-1, keepdims=True), 1e-12)  # F.normalize
    orient, fscale = face_orientation(verts, faces)
    qf, m_f = rotmat_to_unitquat(orient)
    bind = np.asarray(binding_face).astype(np.int64)
    fv = verts[:, np.asarray(faces).astype(np.int64)]  # B,F,3,3
    fvn = fv[:, bind]  # B,N,3,3
    bary = np.asarray(face_bary, np.float64)
    centre = np.einsum("nk,bnkj->bnj", bary, fvn)
    s_n = fscale[:, bind]  # B,N,1
    xyz = np.einsum("bnij,bnj->bni", orient[:, bind], per_frame(local_xyz)) * s_n + centre
    qu = xyzw_to_wxyz(quat_product(qf[:, bind], wxyz_to_xyzw(per_frame(uv_rotations))))
    return dict(xyz=np.concatenate([verts, xyz], 1),
                rotation=np.concatenate([qv, qu], 1),
                scaling=np.concatenate([per_frame(vtx_scales), per_frame(uv_scales) * s_n], 1),
                margin=np.concatenate([m_v, m_f[:, bind]], 1))


def ehm_forward(body, flame, extra, body_params, flame_params):
    """EHM.forward (modules/ehm/EHM.py:36-137) on numpy assets (avatar.ehm_assets layout):
    FLAME head lbs (jaw + eyes; global and neck zeroed, :59-63) + eyelids + head_scale (:72-75),
    body blend_shapes + joints (:114-118), head splice (:121-124), body lbs_wobeta with jaw and eyes
    zeroed (:98-99, :134-137).  Returns dict(vertices, joints, joints_transform, ver_transform_mat,
    joint_transform_mat)."""
    fp, bp = flame_params, body_params
    B = fp["shape_params"].shape[0]
    betas = np.concatenate([fp["shape_params"], fp["expression_params"]], 1)
    zeros3 = np.zeros((B, 3))
    full = np.concatenate([zeros3, zeros3, fp["jaw_params"], fp["eye_pose_params"]], 1)
    hv, hj, *_ = lbs(betas, full, flame["v_template"], flame["shapedirs"], flame["posedirs"],
                     flame["J_regressor"], flame["parents"], flame["lbs_weights"])
    hv = hv + extra["r_eyelid"][None] * np.asarray(fp["eyelid_params"], np.float64)[:, 1:2, None]
    hv = hv + extra["l_eyelid"][None] * np.asarray(fp["eyelid_params"], np.float64)[:, 0:1, None]
    hv = hv * np.asarray(bp["head_scale"], np.float64)[:, None]
    sc = np.concatenate([bp["shape"], bp["exp"]], 1)
    vt = np.asarray(body["v_template"], np.float64) + blend_shapes(sc, body["shapedirs"])
    tj = vertices2joints(body["J_regressor"], vt) + np.asarray(bp["joints_offset"], np.float64)
    idx = np.asarray(extra["smplx2flame_ind"]).astype(np.int64)
    vt[:, idx] = hv - hj[:, 3:5].mean(1, keepdims=True) + tj[:, 23:25].mean(1, keepdims=True)
    pose = np.concatenate([bp["global_pose"].reshape(B, 1, 3), bp["body_pose"], np.zeros((B, 3, 3)),
                           bp["left_hand_pose"], bp["right_hand_pose"]], 1)
    verts, jt, J, T, A = lbs_wobeta(pose, vt, body["posedirs"], body["J_regressor"], body["parents"],
                                    body["lbs_weights"], bp["joints_offset"])
    return dict(vertices=verts, joints=J, joints_transform=jt, ver_transform_mat=T, joint_transform_mat=A)
