"""CPU tests of the deformation oracle (oracle/lbs_oracle.py).

* Pinned against the reference: lbs / lbs_wobeta / batch_rodrigues outputs produced by the
  reference's own models/modules/flame/lbs.py (tests/golden/lbs_golden.npz, make_lbs_golden.py).
  Tolerance 2e-5 absolute (the reference ran in float32 on CPU torch, the oracle in float64).
* roma / compute_face_orientation restatements (not importable here: parity unpinned against the
  reference) are checked by properties: unit quaternions that reproduce the rotation (via an
  independent quaternion->matrix formula and scipy's Rotation), right-handed orthonormal frames,
  Hamilton-product composition.
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(HERE, "golden"))
import lbs_cases  # noqa: E402
import lbs_oracle as lo  # noqa: E402

GOLD = os.path.join(HERE, "golden", "lbs_golden.npz")
ATOL = 2e-5


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


@pytest.fixture(scope="module")
def cases():
    return lbs_cases.all_cases()


def test_golden_inputs_unchanged(gold, cases):
    for name, c in cases.items():
        assert bytes(gold[f"{name}/sha"]).decode() == lbs_cases.digest(c), \
            f"{name}: input generator drifted; rerun tests/golden/make_lbs_golden.py"


def test_rodrigues_matches_reference(gold, cases):
    R = lo.batch_rodrigues(cases["rodrigues"]["rot_vecs"])
    np.testing.assert_allclose(R, gold["rodrigues/rot"], atol=ATOL, rtol=0)


@pytest.mark.parametrize("name", ["smplx_wobeta", "smplx_rotmat"])
def test_lbs_wobeta_matches_reference(gold, cases, name):
    c = cases[name]
    verts, jt, J, T, A = lo.lbs_wobeta(c["pose"], c["v_shaped"], c["posedirs"], c["J_regressor"],
                                       c["parents"], c["lbs_weights"], c["joints_offset"],
                                       c["pose2rot"])
    for key, got in (("verts", verts), ("J_transformed", jt), ("J", J), ("T", T), ("A", A)):
        np.testing.assert_allclose(got, gold[f"{name}/{key}"], atol=ATOL, rtol=0, err_msg=key)


def test_lbs_with_betas_matches_reference(gold, cases):
    c = cases["flame_lbs"]
    verts, jt, *_ = lo.lbs(c["betas"], c["pose"], c["v_template"], c["shapedirs"], c["posedirs"],
                           c["J_regressor"], c["parents"], c["lbs_weights"], c["joints_offset"])
    np.testing.assert_allclose(verts, gold["flame_lbs/verts"], atol=ATOL, rtol=0)
    np.testing.assert_allclose(jt, gold["flame_lbs/J_transformed"], atol=ATOL, rtol=0)


def _quat_to_mat_wxyz(q):
    w, x, y, z = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    return np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                     2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                     2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1).reshape(q.shape[:-1] + (3, 3))


def _random_rotations(n, seed):
    rng = np.random.default_rng(seed)
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    return _quat_to_mat_wxyz(q)


def test_rotmat_to_unitquat_round_trip():
    R = _random_rotations(2000, 0)
    # every decision branch: near-identity, and 180-degree turns about each axis
    R[:4] = np.stack([np.eye(3), np.diag([1.0, -1, -1]), np.diag([-1.0, 1, -1]), np.diag([-1.0, -1, 1])])
    q, _ = lo.rotmat_to_unitquat(R)
    np.testing.assert_allclose(np.linalg.norm(q, axis=1), 1.0, atol=1e-12)
    np.testing.assert_allclose(_quat_to_mat_wxyz(lo.xyzw_to_wxyz(q)), R, atol=1e-12)
    from scipy.spatial.transform import Rotation
    qs = Rotation.from_matrix(R).as_quat()  # xyzw
    err = np.minimum(np.abs(q - qs).max(1), np.abs(q + qs).max(1))
    assert err.max() < 1e-12


def test_quat_product_composes_rotations():
    Ra, Rb = _random_rotations(500, 1), _random_rotations(500, 2)
    qa, _ = lo.rotmat_to_unitquat(Ra)
    qb, _ = lo.rotmat_to_unitquat(Rb)
    qc = lo.quat_product(qa, qb)
    np.testing.assert_allclose(_quat_to_mat_wxyz(lo.xyzw_to_wxyz(qc)), Ra @ Rb, atol=1e-12)


def test_face_orientation_is_right_handed_orthonormal():
    rng = np.random.default_rng(3)
    verts = rng.normal(size=(2, 400, 3))
    faces = np.stack([rng.choice(400, 3, replace=False) for _ in range(300)])
    M, s = lo.face_orientation(verts, faces)
    np.testing.assert_allclose(np.swapaxes(M, -1, -2) @ M, np.broadcast_to(np.eye(3), M.shape), atol=1e-12)
    np.testing.assert_allclose(np.linalg.det(M), 1.0, atol=1e-12)
    e1 = verts[:, faces[:, 1]] - verts[:, faces[:, 0]]
    np.testing.assert_allclose(M[..., 0], e1 / np.linalg.norm(e1, axis=-1, keepdims=True), atol=1e-12)
    assert (s > 0).all()


def test_deform_identity_pose_keeps_gaussians():
    """Identity skinning: vertex Gaussians keep position/rotation/scale; UV Gaussians sit at the
    barycentric point plus the face-frame offset (ubody_gaussian.py:252-271)."""
    rng = np.random.default_rng(4)
    V, F, N, B = 50, 40, 120, 2
    verts = rng.normal(size=(B, V, 3))
    faces = np.stack([rng.choice(V, 3, replace=False) for _ in range(F)])
    T = np.broadcast_to(np.eye(4), (B, V, 4, 4))
    qv = rng.normal(size=(V, 4))
    qv /= np.linalg.norm(qv, axis=1, keepdims=True)
    qv[qv[:, 0] < 0] *= -1
    bind = rng.integers(0, F, N)
    bary = rng.dirichlet([1, 1, 1], N)
    out = lo.deform_gaussians(verts, T, faces, qv, np.ones((V, 3)), bind, bary, np.zeros((N, 3)),
                              np.tile([1.0, 0, 0, 0], (N, 1)), np.ones((N, 3)))
    np.testing.assert_allclose(out["xyz"][:, :V], verts, atol=1e-12)
    q = out["rotation"][:, :V]
    np.testing.assert_allclose(np.minimum(np.abs(q - qv).max(-1), np.abs(q + qv).max(-1)), 0, atol=1e-12)
    centre = np.einsum("nk,bnkj->bnj", bary, verts[:, faces[bind]])
    np.testing.assert_allclose(out["xyz"][:, V:], centre, atol=1e-12)


@pytest.fixture(scope="module")
def full():
    return np.load(os.path.join(HERE, "golden", "lbs_golden_full.npz")), lbs_cases.full_cases()


def test_full_size_lbs_matches_reference(full):
    """SURVEY.md §8(c) sizes: SMPL-X body lbs_wobeta at V = 10,595 (template + 120 teeth), J = 55, and
    the FLAME head lbs at V = 5,023 with 400 betas -- the oracle against the reference's lbs.py."""
    gold, cases = full
    for name, c in cases.items():
        assert bytes(gold[f"{name}/sha"]).decode() == lbs_cases.digest(c), \
            f"{name}: input generator drifted; rerun tests/golden/make_lbs_golden.py"
    c = cases["smplx_full_wobeta"]
    assert c["v_shaped"].shape[1] == 10595 and c["J_regressor"].shape[0] == 55
    out = lo.lbs_wobeta(c["pose"], c["v_shaped"], c["posedirs"], c["J_regressor"], c["parents"],
                        c["lbs_weights"], c["joints_offset"], c["pose2rot"])
    for key, got in zip(("verts", "J_transformed", "J", "T", "A"), out):
        np.testing.assert_allclose(got, gold[f"smplx_full_wobeta/{key}"], atol=ATOL, rtol=0, err_msg=key)
    c = cases["flame_full_lbs"]
    verts, jt, *_ = lo.lbs(c["betas"], c["pose"], c["v_template"], c["shapedirs"], c["posedirs"],
                           c["J_regressor"], c["parents"], c["lbs_weights"], c["joints_offset"])
    np.testing.assert_allclose(verts, gold["flame_full_lbs/verts"], atol=ATOL, rtol=0)
    np.testing.assert_allclose(jt, gold["flame_full_lbs/J_transformed"], atol=ATOL, rtol=0)
