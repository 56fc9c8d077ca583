"""Synthetic GUAVA avatar assets (numpy float32): SMPL-X-shaped LBS model + vertex/UV Gaussians.

The licensed SMPL-X / FLAME model files and the pretrained GUAVA checkpoint are not available
offline, so the deformation path is exercised on assets with the reference's
shapes and structure:

  * mesh: the SMPL-X template vertices and faces shipped with the reference
    (assets/SMPLX/smplx_uv.obj, smplx_faces.npy -> tests/golden/avatar_template.npz), turned to face
    the canonical camera as in scenes.avatar_cloud;
  * kinematic tree: SMPL-X's 55 joints (1 global + 21 body + jaw + 2 eyes + 2 x 15 hand) with the
    SMPL-X parent order (parents[i] < i, as batch_rigid_transform requires, lbs.py:462-468);
  * J_regressor [J,V]: each joint the normalised mean of its 8 nearest template vertices;
  * lbs_weights [V,J]: softmax over the 4 nearest joints (rows sum to 1);
  * shapedirs [V,3,NB] / posedirs [9(J-1), 3V]: small Gaussian bases (NB = 300 shape + 50
    expression components as EHM.forward concatenates them, EHM.py:106);
  * Gaussians: one per template vertex (vertex Gaussians, ubody_gaussian.py:169-173) and one per
    covered UV texel of assets/SMPLX/uv_masks/uv_mask512_with_faceid_smplx.npy bound to its face
    at a random barycentric point (UV Gaussians, :175-182), pruned at random to P, with GUAVA's
    decoder distributions (feature_decoder.py:52-58,123-129; see scenes.py).
"""
import numpy as np

from . import scenes

C = 32
# SMPL-X kinematic tree (55 joints)
SMPLX_PARENTS = np.array([-1, 0, 0, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 9, 9, 12, 13, 14, 16, 17, 18, 19,
                          15, 15, 15, 20, 25, 26, 20, 28, 29, 20, 31, 32, 20, 34, 35, 20, 37, 38,
                          21, 40, 41, 21, 43, 44, 21, 46, 47, 21, 49, 50, 21, 52, 53], np.int32)
# FLAME kinematic tree (global, neck, jaw, left eye, right eye)
FLAME_PARENTS = np.array([-1, 0, 1, 1, 1], np.int32)


def template_mesh():
    """(verts [V,3] f32 in the camera-facing frame, faces [F,3] i32, texel_count [F] i64)."""
    fx = np.load(scenes._FIXTURE)
    v = fx["verts"].astype(np.float32)
    v = np.stack([v[:, 0], -v[:, 1] - 0.85, -v[:, 2]], 1).astype(np.float32)
    return v, fx["faces"].astype(np.int32), fx["texel_count"].astype(np.int64)


def lbs_model(verts, J=55, NB=350, parents=None, seed=0, shape_scale=2e-4, pose_scale=1e-3):
    """SMPL-X-shaped LBS assets on the given template (reference layouts, float32)."""
    rng = np.random.default_rng(seed)
    V = verts.shape[0]
    parents = SMPLX_PARENTS if parents is None else np.asarray(parents, np.int32)
    assert parents.shape[0] == J
    # joint centres: a spatially coherent tree -- the root at the vertex nearest the centroid, each
    # child a random vertex 8-20 cm from its parent joint (so a joint rotation moves nearby skin)
    centres = np.empty((J, 3), np.float32)
    centres[0] = verts[int(np.argmin(((verts - verts.mean(0)) ** 2).sum(1)))]
    for j in range(1, J):
        d = np.sqrt(((verts - centres[parents[j]]) ** 2).sum(1))
        cand = np.nonzero((d > 0.08) & (d < 0.2))[0]
        if cand.size == 0:
            cand = np.argsort(d)[: max(1, V // 10)]
        centres[j] = verts[int(rng.choice(cand))]
    d2 = ((verts[:, None, :] - centres[None]) ** 2).sum(-1)  # V,J
    jreg = np.zeros((J, V), np.float32)
    near_v = np.argsort(d2, axis=0)[:8]  # 8 nearest vertices per joint
    for j in range(J):
        jreg[j, near_v[:, j]] = 1.0 / 8.0
    near_j = np.argsort(d2, axis=1)[:, :4]
    logits = -np.take_along_axis(d2, near_j, 1) / max(float(np.median(d2)) * 0.01, 1e-6)
    logits -= logits.max(1, keepdims=True)
    w4 = np.exp(logits)
    w4 /= w4.sum(1, keepdims=True)
    weights = np.zeros((V, J), np.float32)
    np.put_along_axis(weights, near_j, w4.astype(np.float32), 1)
    shapedirs = (rng.normal(size=(V, 3, NB)) * shape_scale).astype(np.float32) if NB else None
    posedirs = (rng.normal(size=(9 * (J - 1), 3 * V)) * pose_scale).astype(np.float32)
    return dict(v_template=verts.astype(np.float32), shapedirs=shapedirs, posedirs=posedirs,
                J_regressor=jreg, parents=parents, lbs_weights=weights)


def random_pose(B, J=55, sigma=0.15, seed=1000, body_joints=range(1, 22)):
    """Axis-angle poses [B,J,3]: N(0, sigma) on the body joints, zero elsewhere;
    frame b uses seed + b."""
    out = np.zeros((B, J, 3), np.float32)
    for b in range(B):
        rng = np.random.default_rng(seed + b)
        for j in body_joints:
            if j < J:
                out[b, j] = rng.normal(0.0, sigma, 3)
    return out


def gaussians(verts, faces, texel_count, P=100000, seed=0):
    """Canonical vertex + UV Gaussian assets (Ubody_Gaussian's inputs, ubody_gaussian.py:169-187).
    All V vertex Gaussians are kept; UV Gaussians are pruned at random so that V + N = P."""
    rng = np.random.default_rng(seed)
    V = verts.shape[0]
    face_of = np.repeat(np.arange(faces.shape[0]), texel_count)
    N = max(0, min(P - V, face_of.shape[0]))
    keep = np.sort(rng.choice(face_of.shape[0], N, replace=False))
    bind = face_of[keep].astype(np.int32)
    bary = rng.dirichlet([1.0, 1.0, 1.0], N).astype(np.float32)
    local = rng.normal(0.0, 0.2, (N, 3)).astype(np.float32)

    def unit_quats(n):
        q = rng.normal(size=(n, 4)).astype(np.float32)
        return (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)

    def feats(n):
        f = np.empty((n, C), np.float32)
        f[:, :3] = rng.uniform(0.0, 1.0, (n, 3))
        f[:, 3:] = rng.normal(size=(n, C - 3))
        return f

    def opac(n):
        o = (1.0 / (1.0 + np.exp(-rng.normal(0.0, 1.5, n)))).astype(np.float32)
        return np.maximum(o, np.float32(0.0011)).reshape(n, 1)

    return dict(
        vtx_rotations=unit_quats(V),
        vtx_scales=(0.05 / (1.0 + np.exp(-rng.normal(size=(V, 3))))).astype(np.float32),
        binding_face=bind, face_bary=bary, local_xyz=local, uv_rotations=unit_quats(N),
        uv_scales=np.exp(rng.normal(-0.7, 0.3, (N, 3))).astype(np.float32),
        opacities=np.concatenate([opac(V), opac(N)], 0),
        colors=np.concatenate([feats(V), feats(N)], 0))


def ehm_assets(seed=0, n_shape=300, n_exp=50):
    """SMPL-X body + FLAME head LBS assets wired as EHM (modules/ehm/EHM.py:14-34): the FLAME
    template is the SMPL-X template's FLAME-mapped region (SMPL-X__FLAME_vertex_ids.npy), the
    eyelid blend shapes are the reference's flame_{l,r}_eyelid.npy.  Returns (body, flame, extra)."""
    fx = np.load(scenes._FIXTURE)
    verts, faces, _ = template_mesh()
    nb = n_shape + n_exp
    body = lbs_model(verts, J=55, NB=nb, parents=SMPLX_PARENTS, seed=seed)
    idx = fx["smplx2flame_ind"].astype(np.int32)
    flame = lbs_model(verts[idx], J=5, NB=nb, parents=FLAME_PARENTS, seed=seed + 1)
    # the splice re-anchors the head from FLAME joints 3:5 to body joints 23:25 (EHM.py:123): regress
    # the body's 23, 24 from the same (mapped) vertices so the head stays on the neck at rest
    for jb, jh in ((23, 3), (24, 4)):
        body["J_regressor"][jb] = 0.0
        np.add.at(body["J_regressor"][jb], idx, flame["J_regressor"][jh])
    extra = dict(smplx2flame_ind=idx, l_eyelid=fx["l_eyelid"].astype(np.float32),
                 r_eyelid=fx["r_eyelid"].astype(np.float32), faces=faces)
    return body, flame, extra


def ehm_params(B, seed=1000, n_shape=300, n_exp=50, body_sigma=0.15):
    """Per-frame EHM inputs (the keys EHM.forward reads, EHM.py:42-91) for B tracked frames: a fixed
    identity (shape), per-frame expression / jaw / eyes / eyelids / body and hand poses."""
    rng = np.random.default_rng(seed)
    shape = np.broadcast_to(rng.normal(0, 1, (1, n_shape)), (B, n_shape)).astype(np.float32)
    f = lambda *s: rng.normal(0, 1, s).astype(np.float32)  # noqa: E731
    body = dict(shape=shape.copy(), exp=0.5 * f(B, n_exp),
                global_pose=0.05 * f(B, 1, 3), body_pose=random_pose(B, J=22, sigma=body_sigma, seed=seed)[:, 1:],
                left_hand_pose=0.2 * f(B, 15, 3), right_hand_pose=0.2 * f(B, 15, 3),
                joints_offset=0.002 * f(B, 55, 3),
                head_scale=(1.0 + 0.02 * f(B, 3)).astype(np.float32))
    flame = dict(shape_params=shape.copy(), expression_params=0.5 * f(B, n_exp),
                 pose_params=0.05 * f(B, 3), jaw_params=0.1 * np.abs(f(B, 3)),
                 eye_pose_params=0.05 * f(B, 6),
                 eyelid_params=np.clip(0.5 + 0.2 * f(B, 2), 0.0, 1.0).astype(np.float32))
    return body, flame


def change_id_info(target_body, target_flame, source_body, source_flame):
    """Cross-reenactment inputs (main/test.py:21-28 change_id_info): the target frames' pose and
    expression with the SOURCE identity -- shape, joints_offset, head_scale and the FLAME shape come
    from the source (its first frame, broadcast over the target's B frames).  hand_scale is not part
    of these assets (EHMDeformer rejects it: the MANO vertex map is not bundled)."""
    B = target_flame["shape_params"].shape[0]
    body = dict(target_body)
    flame = dict(target_flame)
    for k in ("shape", "joints_offset", "head_scale"):
        if source_body.get(k) is not None:
            body[k] = np.ascontiguousarray(np.broadcast_to(source_body[k][:1], (B,) + source_body[k].shape[1:]))
    flame["shape_params"] = np.ascontiguousarray(
        np.broadcast_to(source_flame["shape_params"][:1], (B,) + source_flame["shape_params"].shape[1:]))
    return body, flame
