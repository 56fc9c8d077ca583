"""Deterministic synthetic inputs of the LBS golden cases (used by make_lbs_golden.py and the tests).

Shapes follow the reference's callers: SMPL-X body lbs_wobeta (EHM.py:134-137, 55 joints) and the
FLAME head lbs (EHM.py:67-70, 5 joints, shape+expression betas), on subsets of the SMPL-X template
shipped with the reference (tests/golden/avatar_template.npz).
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
from guava_renderer_amd import avatar  # noqa: E402


def _subset(n, seed):
    verts, _, _ = avatar.template_mesh()
    idx = np.sort(np.random.default_rng(seed).choice(verts.shape[0], n, replace=False))
    return verts[idx]


def all_cases():
    cases = {}
    # SMPL-X body: lbs_wobeta, axis-angle, joints_offset, B=3
    rng = np.random.default_rng(11)
    m = avatar.lbs_model(_subset(300, 1), J=55, NB=0, seed=2, pose_scale=2e-3)
    B = 3
    pose = rng.normal(0.0, 0.3, (B, 55, 3)).astype(np.float32)
    v_shaped = (m["v_template"][None] + rng.normal(0.0, 0.01, (B, 300, 3))).astype(np.float32)
    cases["smplx_wobeta"] = dict(kind="lbs_wobeta", B=B, pose=pose, v_shaped=v_shaped,
                                 posedirs=m["posedirs"], J_regressor=m["J_regressor"],
                                 parents=m["parents"], lbs_weights=m["lbs_weights"],
                                 joints_offset=rng.normal(0.0, 0.01, (B, 55, 3)).astype(np.float32),
                                 pose2rot=True)
    # SMPL-X body, rotation-matrix pose (pose2rot=False), B=2, no offset
    rng = np.random.default_rng(12)
    m = avatar.lbs_model(_subset(150, 3), J=55, NB=0, seed=4)
    aa = rng.normal(0.0, 0.5, (2 * 55, 3))
    ang = np.linalg.norm(aa, axis=1, keepdims=True)
    k = aa / ang
    K = np.zeros((aa.shape[0], 3, 3))
    K[:, 0, 1], K[:, 0, 2], K[:, 1, 0] = -k[:, 2], k[:, 1], k[:, 2]
    K[:, 1, 2], K[:, 2, 0], K[:, 2, 1] = -k[:, 0], -k[:, 1], k[:, 0]
    R = np.eye(3) + np.sin(ang)[:, :, None] * K + (1 - np.cos(ang))[:, :, None] * (K @ K)
    cases["smplx_rotmat"] = dict(kind="lbs_wobeta", B=2, pose=R.reshape(2, 55, 3, 3).astype(np.float32),
                                 v_shaped=np.broadcast_to(m["v_template"], (2, 150, 3)).copy(),
                                 posedirs=m["posedirs"], J_regressor=m["J_regressor"],
                                 parents=m["parents"], lbs_weights=m["lbs_weights"],
                                 joints_offset=None, pose2rot=False)
    # FLAME head: lbs with betas (shape + expression), 5 joints, B=2
    rng = np.random.default_rng(13)
    m = avatar.lbs_model(_subset(200, 5), J=5, NB=24, parents=avatar.FLAME_PARENTS, seed=6,
                         shape_scale=5e-3)
    cases["flame_lbs"] = dict(kind="lbs", B=2, betas=rng.normal(0.0, 1.0, (2, 24)).astype(np.float32),
                              pose=rng.normal(0.0, 0.3, (2, 5 * 3)).astype(np.float32),
                              v_template=m["v_template"], shapedirs=m["shapedirs"],
                              posedirs=m["posedirs"], J_regressor=m["J_regressor"],
                              parents=m["parents"], lbs_weights=m["lbs_weights"],
                              joints_offset=None, pose2rot=True)
    # batch_rodrigues edge cases: zero, tiny, pi, large, negative
    rng = np.random.default_rng(14)
    rv = rng.normal(0.0, 1.0, (64, 3)).astype(np.float32)
    rv[0] = 0.0
    rv[1] = [1e-9, 0.0, 0.0]
    rv[2] = [np.pi, 0.0, 0.0]
    rv[3] = [0.0, -np.pi, 0.0]
    rv[4] = [3.0, 4.0, -5.0]
    rv[5] = [-1e-4, 2e-4, -3e-4]
    cases["rodrigues"] = dict(kind="rodrigues", rot_vecs=rv)
    return cases


def _teeth_template(n_teeth=120, seed=31):
    """SMPL-X template (10,475 vertices) + 120 teeth vertices, the V = 10,595 of EHM's body mesh
    (SMPLX.py:470-481 appends the teeth): synthetic teeth near the mouth region (the template's
    front-most head vertices, jittered by 2 mm)."""
    verts, _, _ = avatar.template_mesh()
    rng = np.random.default_rng(seed)
    head = np.nonzero(verts[:, 1] > np.percentile(verts[:, 1], 92))[0]
    front = head[np.argsort(-verts[head, 2])[: 4 * n_teeth]]
    pick = rng.choice(front, n_teeth, replace=False)
    teeth = verts[pick] + rng.normal(0.0, 0.002, (n_teeth, 3))
    return np.concatenate([verts, teeth]).astype(np.float32)


def full_cases():
    """SURVEY.md §8(c)'s full-size cases: SMPL-X body lbs_wobeta at V = 10,595, J = 55 (B = 2,
    axis-angle pose, joints_offset) and the FLAME head lbs at FLAME size (V = 5,023, J = 5, 400
    shape + expression betas, B = 2).  The inputs (62 MB of posedirs) are regenerated from the seeds;
    lbs_golden_full.npz keeps the reference's outputs and the inputs' SHA-256."""
    cases = {}
    rng = np.random.default_rng(41)
    verts = _teeth_template()
    m = avatar.lbs_model(verts, J=55, NB=0, seed=42, pose_scale=1e-3)
    B, V = 2, verts.shape[0]
    assert V == 10595
    cases["smplx_full_wobeta"] = dict(
        kind="lbs_wobeta", B=B, pose=rng.normal(0.0, 0.3, (B, 55, 3)).astype(np.float32),
        v_shaped=(m["v_template"][None] + rng.normal(0.0, 0.005, (B, V, 3))).astype(np.float32),
        posedirs=m["posedirs"], J_regressor=m["J_regressor"], parents=m["parents"],
        lbs_weights=m["lbs_weights"], joints_offset=rng.normal(0.0, 0.01, (B, 55, 3)).astype(np.float32),
        pose2rot=True)
    rng = np.random.default_rng(43)
    m = avatar.lbs_model(_subset(5023, 44), J=5, NB=400, parents=avatar.FLAME_PARENTS, seed=45,
                         shape_scale=2e-4)
    cases["flame_full_lbs"] = dict(kind="lbs", B=2, betas=rng.normal(0.0, 1.0, (2, 400)).astype(np.float32),
                                   pose=rng.normal(0.0, 0.3, (2, 5 * 3)).astype(np.float32),
                                   v_template=m["v_template"], shapedirs=m["shapedirs"],
                                   posedirs=m["posedirs"], J_regressor=m["J_regressor"],
                                   parents=m["parents"], lbs_weights=m["lbs_weights"],
                                   joints_offset=None, pose2rot=True)
    return cases


def digest(case):
    h = hashlib.sha256()
    for k in sorted(case):
        v = case[k]
        if isinstance(v, np.ndarray):
            h.update(k.encode())
            h.update(np.ascontiguousarray(v).tobytes())
        else:
            h.update(f"{k}={v!r}".encode())
    return h.hexdigest()
