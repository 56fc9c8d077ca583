"""GPU parity of the deformation path (csrc/deform.hip via include/gsr_deform.h) against the CPU
oracle (oracle/lbs_oracle.py, itself pinned to the reference's lbs.py in test_lbs_oracle.py).

Tolerances (float32 GPU vs float64 oracle):
  vertices, joints, transforms  2e-5 absolute (coordinates are O(1))
  Gaussian means / scales       2e-5 absolute
  quaternions                   2e-5 absolute up to sign, on Gaussians whose rotmat_to_unitquat
                                decision margin is >= 1e-4 (below it float32 may take another
                                branch of the decision scheme, which the test counts separately)
Indices (faces, binding faces) are integers: the gathered vertices must be the oracle's exactly,
which the 2e-5 bound on UV means checks.
"""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import lbs_cases  # noqa: E402
import lbs_oracle as lo  # noqa: E402

pytestmark = pytest.mark.gpu
ATOL = 2e-5
DEV = "cuda:0"


def _t(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(DEV) if x is not None else None


def _gpu_wobeta(c):
    from guava_renderer_amd import deform
    out = deform.lbs_wobeta(_t(c["pose"]), _t(c["v_shaped"]), _t(c["posedirs"]), _t(c["J_regressor"]),
                            torch.from_numpy(c["parents"]), _t(c["lbs_weights"]),
                            joints_offset=_t(c["joints_offset"]), pose2rot=c["pose2rot"])
    return [o.cpu().numpy() for o in out]


@pytest.mark.parametrize("name", ["smplx_wobeta", "smplx_rotmat"])
def test_lbs_wobeta_golden_cases(name):
    c = lbs_cases.all_cases()[name]
    got = _gpu_wobeta(c)
    ref = lo.lbs_wobeta(c["pose"], c["v_shaped"], c["posedirs"], c["J_regressor"], c["parents"],
                        c["lbs_weights"], c["joints_offset"], c["pose2rot"])
    for key, g, r in zip(("verts", "J_transformed", "J", "T", "A"), got, ref):
        np.testing.assert_allclose(g, r, atol=ATOL, rtol=0, err_msg=key)


def test_lbs_with_betas_golden_case():
    from guava_renderer_amd import deform
    c = lbs_cases.all_cases()["flame_lbs"]
    verts, jt = deform.lbs(_t(c["betas"]), _t(c["pose"]), _t(c["v_template"]), _t(c["shapedirs"]),
                           _t(c["posedirs"]), _t(c["J_regressor"]), torch.from_numpy(c["parents"]),
                           _t(c["lbs_weights"]))
    r_verts, r_jt, *_ = lo.lbs(c["betas"], c["pose"], c["v_template"], c["shapedirs"], c["posedirs"],
                               c["J_regressor"], c["parents"], c["lbs_weights"])
    np.testing.assert_allclose(verts.cpu().numpy(), r_verts, atol=ATOL, rtol=0)
    np.testing.assert_allclose(jt.cpu().numpy(), r_jt, atol=ATOL, rtol=0)


@pytest.fixture(scope="module")
def full_golden():
    return np.load(os.path.join(HERE, "golden", "lbs_golden_full.npz")), lbs_cases.full_cases()


@pytest.mark.parametrize("frames", [(0, 1), (1,)])
def test_full_size_goldens_match_reference(full_golden, frames):
    """The GPU LBS at SURVEY.md §8(c)'s sizes against the reference's own lbs.py outputs
    (lbs_golden_full.npz): SMPL-X lbs_wobeta at V = 10,595, J = 55 and FLAME lbs at V = 5,023 with
    400 betas; both frames as one batch, and frame 1 alone (B = 1: the single-frame blend kernel)."""
    from guava_renderer_amd import deform
    gold, cases = full_golden
    sel = list(frames)
    c = cases["smplx_full_wobeta"]
    got = deform.lbs_wobeta(_t(c["pose"][sel]), _t(c["v_shaped"][sel]), _t(c["posedirs"]), _t(c["J_regressor"]),
                            torch.from_numpy(c["parents"]), _t(c["lbs_weights"]),
                            joints_offset=_t(c["joints_offset"][sel]), pose2rot=True)
    for key, g in zip(("verts", "J_transformed", "J", "T", "A"), got):
        np.testing.assert_allclose(g.cpu().numpy(), gold[f"smplx_full_wobeta/{key}"][sel], atol=ATOL, rtol=0,
                                   err_msg=key)
    c = cases["flame_full_lbs"]
    verts, jt = deform.lbs(_t(c["betas"][sel]), _t(c["pose"][sel]), _t(c["v_template"]), _t(c["shapedirs"]),
                           _t(c["posedirs"]), _t(c["J_regressor"]), torch.from_numpy(c["parents"]),
                           _t(c["lbs_weights"]))
    np.testing.assert_allclose(verts.cpu().numpy(), gold["flame_full_lbs/verts"][sel], atol=ATOL, rtol=0)
    np.testing.assert_allclose(jt.cpu().numpy(), gold["flame_full_lbs/J_transformed"][sel], atol=ATOL, rtol=0)


def test_single_frame_deform_matches_oracle():
    """B = 1 everywhere (the per-frame drop-in path, main/test.py:70-76): lbs with betas and
    posedirs at SMPL-X size, lbs_wobeta, and EHM.forward, each against the oracle -- the
    single-frame blend kernel (k_lbs_blend<1,16>) and its scalar tail for NF % 4 != 0."""
    from guava_renderer_amd import avatar, deform
    m, g, faces, betas, pose = _full_avatar(B=1, P=20000)
    verts, jt = deform.lbs(_t(betas), _t(pose), _t(m["v_template"]), _t(m["shapedirs"]), _t(m["posedirs"]),
                           _t(m["J_regressor"]), torch.from_numpy(m["parents"]), _t(m["lbs_weights"]))
    r_verts, r_jt, r_J, r_T, r_A, r_vs = lo.lbs(betas, pose, m["v_template"], m["shapedirs"], m["posedirs"],
                                                m["J_regressor"], m["parents"], m["lbs_weights"])
    np.testing.assert_allclose(verts.cpu().numpy(), r_verts, atol=ATOL, rtol=0)
    np.testing.assert_allclose(jt.cpu().numpy(), r_jt, atol=ATOL, rtol=0)
    _, _, _, T2, A2 = deform.lbs_wobeta(_t(pose), _t(r_vs.astype(np.float32)), _t(m["posedirs"]),
                                        _t(m["J_regressor"]), torch.from_numpy(m["parents"]), _t(m["lbs_weights"]))
    np.testing.assert_allclose(T2.cpu().numpy(), r_T, atol=ATOL, rtol=0)
    np.testing.assert_allclose(A2.cpu().numpy(), r_A, atol=ATOL, rtol=0)
    # a blend with a coefficient count that is not a multiple of 4 (the scalar tail): 350 - 3 betas
    nb = 347
    v3, _ = deform.lbs(_t(betas[:, :nb]), _t(pose), _t(m["v_template"]), _t(m["shapedirs"][..., :nb].copy()),
                       _t(m["posedirs"]), _t(m["J_regressor"]), torch.from_numpy(m["parents"]),
                       _t(m["lbs_weights"]))
    r3, *_ = lo.lbs(betas[:, :nb], pose, m["v_template"], m["shapedirs"][..., :nb], m["posedirs"],
                    m["J_regressor"], m["parents"], m["lbs_weights"])
    np.testing.assert_allclose(v3.cpu().numpy(), r3, atol=ATOL, rtol=0)
    body, flame, extra = avatar.ehm_assets(seed=0)
    bp, fp = avatar.ehm_params(1, seed=4000)
    ehm = deform.EHMDeformer(body, flame, extra["smplx2flame_ind"], extra["l_eyelid"], extra["r_eyelid"],
                             device=DEV)
    out = ehm({k: _t(v) for k, v in bp.items()}, {k: _t(v) for k, v in fp.items()})
    ref = lo.ehm_forward(body, flame, extra, bp, fp)
    for k in ("vertices", "joints", "joints_transform", "ver_transform_mat", "joint_transform_mat"):
        np.testing.assert_allclose(out[k].cpu().numpy(), ref[k], atol=ATOL, rtol=0, err_msg=k)


def _full_avatar(B=4, P=40000):
    from guava_renderer_amd import avatar
    verts, faces, tex = avatar.template_mesh()
    m = avatar.lbs_model(verts, J=55, NB=350, seed=0)
    g = avatar.gaussians(verts, faces, tex, P=P, seed=0)
    rng = np.random.default_rng(7)
    betas = rng.normal(size=(B, 350)).astype(np.float32)
    pose = avatar.random_pose(B, seed=1000)
    return m, g, faces, betas, pose


def test_full_smplx_lbs_and_gaussian_assembly():
    """SMPL-X size (V=10,475, J=55, NB=350 shape+expression), B=4 frames: lbs -> Gaussians."""
    from guava_renderer_amd import deform
    m, g, faces, betas, pose = _full_avatar()
    B = betas.shape[0]
    # body LBS with betas (EHM.forward = blend_shapes + lbs_wobeta, EHM.py:115,134-137)
    verts, jt = deform.lbs(_t(betas), _t(pose), _t(m["v_template"]), _t(m["shapedirs"]), _t(m["posedirs"]),
                           _t(m["J_regressor"]), torch.from_numpy(m["parents"]), _t(m["lbs_weights"]))
    r_verts, r_jt, r_J, r_T, r_A, r_vs = lo.lbs(betas, pose, m["v_template"], m["shapedirs"], m["posedirs"],
                                                m["J_regressor"], m["parents"], m["lbs_weights"])
    np.testing.assert_allclose(verts.cpu().numpy(), r_verts, atol=ATOL, rtol=0)
    np.testing.assert_allclose(jt.cpu().numpy(), r_jt, atol=ATOL, rtol=0)
    # vertex transforms from lbs_wobeta on the oracle's v_shaped
    v2, jt2, J2, T2, A2 = deform.lbs_wobeta(_t(pose), _t(r_vs.astype(np.float32)), _t(m["posedirs"]),
                                            _t(m["J_regressor"]), torch.from_numpy(m["parents"]),
                                            _t(m["lbs_weights"]))
    np.testing.assert_allclose(T2.cpu().numpy(), r_T, atol=ATOL, rtol=0)
    np.testing.assert_allclose(A2.cpu().numpy(), r_A, atol=ATOL, rtol=0)

    dfm = deform.GaussianDeformer(
        {"rotations": _t(g["vtx_rotations"]), "scales": _t(g["vtx_scales"]),
         "opacities": _t(g["opacities"][:10475]), "colors": _t(g["colors"][:10475])},
        {"rotations": _t(g["uv_rotations"]), "scales": _t(g["uv_scales"]),
         "opacities": _t(g["opacities"][10475:]), "colors": _t(g["colors"][10475:]),
         "local_pos": _t(g["local_xyz"]), "binding_face": _t(g["binding_face"]),
         "face_bary": _t(g["face_bary"])}, _t(faces))
    out = dfm(v2, T2)
    assert not dfm.bad_index()
    ref = lo.deform_gaussians(v2.cpu().numpy(), T2.cpu().numpy(), faces, g["vtx_rotations"],
                              g["vtx_scales"], g["binding_face"], g["face_bary"], g["local_xyz"],
                              g["uv_rotations"], g["uv_scales"])
    np.testing.assert_allclose(out["xyz"].cpu().numpy(), ref["xyz"], atol=ATOL, rtol=0)
    np.testing.assert_allclose(out["scaling"].cpu().numpy(), ref["scaling"], atol=ATOL, rtol=0)
    q, rq = out["rotation"].cpu().numpy(), ref["rotation"]
    err = np.minimum(np.abs(q - rq).max(-1), np.abs(q + rq).max(-1))
    firm = ref["margin"] >= 1e-4
    assert firm.mean() > 0.99
    assert err[firm].max() < ATOL, err[firm].max()
    assert out["opacity"].shape == (B, 40000, 1) and out["features_color"].shape == (B, 40000, 32)


def test_bad_binding_index_is_flagged_not_faulted():
    from guava_renderer_amd import deform
    rng = np.random.default_rng(0)
    V, F, N = 30, 20, 64
    faces = np.stack([rng.choice(V, 3, replace=False) for _ in range(F)]).astype(np.int32)
    bind = rng.integers(0, F, N).astype(np.int32)
    bind[5] = F + 7  # out of range
    q = np.tile(np.array([1, 0, 0, 0], np.float32), (N, 1))
    dfm = deform.GaussianDeformer(
        {"rotations": _t(np.tile(np.array([1, 0, 0, 0], np.float32), (V, 1))),
         "scales": _t(np.ones((V, 3), np.float32)), "opacities": _t(np.ones((V, 1), np.float32)),
         "colors": _t(np.zeros((V, 32), np.float32))},
        {"rotations": _t(q), "scales": _t(np.ones((N, 3), np.float32)),
         "opacities": _t(np.ones((N, 1), np.float32)), "colors": _t(np.zeros((N, 32), np.float32)),
         "local_pos": _t(np.zeros((N, 3), np.float32)), "binding_face": _t(bind),
         "face_bary": _t(np.full((N, 3), 1 / 3, np.float32))}, _t(faces))
    verts = _t(rng.normal(size=(1, V, 3)).astype(np.float32))
    T = _t(np.broadcast_to(np.eye(4, dtype=np.float32), (1, V, 4, 4)))
    out = dfm(verts, T)
    assert dfm.bad_index()
    xyz = out["xyz"].cpu().numpy()
    assert np.isnan(xyz[0, V + 5]).all() and np.isfinite(np.delete(xyz[0], V + 5, 0)).all()


def test_ehm_forward_then_gaussians_match_oracle():
    """EHM.forward (FLAME head lbs + eyelids + head scale + splice + SMPL-X body lbs) for B=3
    frames, then Ubody_Gaussian's assembly, against the oracle composition."""
    from guava_renderer_amd import avatar, deform
    body, flame, extra = avatar.ehm_assets(seed=0)
    bp, fp = avatar.ehm_params(3, seed=1000)
    ehm = deform.EHMDeformer(body, flame, extra["smplx2flame_ind"], extra["l_eyelid"], extra["r_eyelid"],
                             device=DEV)
    out = ehm({k: _t(v) for k, v in bp.items()}, {k: _t(v) for k, v in fp.items()})
    ref = lo.ehm_forward(body, flame, extra, bp, fp)
    for k in ("vertices", "joints", "joints_transform", "ver_transform_mat", "joint_transform_mat"):
        np.testing.assert_allclose(out[k].cpu().numpy(), ref[k], atol=ATOL, rtol=0, err_msg=k)
    assert int(ehm.bad.item()) == 0


def test_ehm_sparse_assets_match_dense(monkeypatch):
    """EHMDeformer's sparse J_regressor (CSR) and skinning weights (K pairs per vertex) against the
    dense kernels (GSR_LBS_SPARSE=0) at B = 1 and B = 5: the joints re-associate their sums
    (1e-6), everything else follows within 2e-6; and both match the oracle."""
    from guava_renderer_amd import avatar, deform
    body, flame, extra = avatar.ehm_assets(seed=0)
    for B in (1, 5):
        bp, fp = avatar.ehm_params(B, seed=5000 + B)
        outs = {}
        for mode in ("1", "0"):
            monkeypatch.setenv("GSR_LBS_SPARSE", mode)
            ehm = deform.EHMDeformer(body, flame, extra["smplx2flame_ind"], extra["l_eyelid"], extra["r_eyelid"],
                                     device=DEV)
            assert bool(ehm.sparse) == (mode == "1")
            if mode == "1":
                assert ehm.sparse["body"][0].skin_k > 0  # the synthetic weights are sparse (<= 4 per vertex)
            outs[mode] = {k: v.cpu().numpy() for k, v in
                          ehm({k: _t(v) for k, v in bp.items()}, {k: _t(v) for k, v in fp.items()}).items()}
        for k in ("vertices", "joints", "joints_transform", "ver_transform_mat", "joint_transform_mat"):
            np.testing.assert_allclose(outs["1"][k], outs["0"][k], atol=2e-6, rtol=0, err_msg=k)
        ref = lo.ehm_forward(body, flame, extra, bp, fp)
        for k in ("vertices", "ver_transform_mat"):
            np.testing.assert_allclose(outs["1"][k], ref[k], atol=ATOL, rtol=0, err_msg=k)


def test_ehm_one_call_equals_per_step_calls():
    """gsr_ehm_forward (one C call, table built in C) against the same steps issued from Python
    (EHMDeformer.forward_calls): the same kernels, so bit-identical outputs -- at B = 1 (the per-frame
    drop-in) and B = 5 with a broadcast head_scale and joints_offset (expanded in the workspace)."""
    from guava_renderer_amd import avatar, deform
    body, flame, extra = avatar.ehm_assets(seed=0)
    ehm = deform.EHMDeformer(body, flame, extra["smplx2flame_ind"], extra["l_eyelid"], extra["r_eyelid"],
                             device=DEV)
    assert ehm.one_call
    for B in (1, 5):
        bp, fp = avatar.ehm_params(B, seed=7000 + B)
        gbp = {k: _t(v) for k, v in bp.items()}
        gfp = {k: _t(v) for k, v in fp.items()}
        if B > 1:
            gbp["head_scale"] = _t(bp["head_scale"][:1])
            gbp["joints_offset"] = _t(np.random.default_rng(B).normal(0, 0.01, (1, 55, 3)).astype(np.float32))
        one = {k: v.cpu().numpy() for k, v in ehm.forward(gbp, gfp).items()}
        if B > 1:  # the per-step path wants joints_offset per frame
            gbp["joints_offset"] = gbp["joints_offset"].expand(B, -1, -1).contiguous()
        steps = {k: v.cpu().numpy() for k, v in ehm.forward_calls(gbp, gfp).items()}
        for k in ("vertices", "joints", "joints_transform", "ver_transform_mat", "joint_transform_mat"):
            np.testing.assert_array_equal(one[k], steps[k], err_msg=f"B={B} {k}")


def test_ehm_forward_large_batch_matrix_core_blend():
    """B=40 frames: the blend shapes run on the matrix-core kernel (k_lbs_blend_mfma, more than 16
    frames), one full 32-frame tile and one partial tile; V*3 = 31,425 is not a multiple of the
    32-coordinate tile either."""
    from guava_renderer_amd import avatar, deform
    body, flame, extra = avatar.ehm_assets(seed=0)
    bp, fp = avatar.ehm_params(40, seed=2000)
    ehm = deform.EHMDeformer(body, flame, extra["smplx2flame_ind"], extra["l_eyelid"], extra["r_eyelid"],
                             device=DEV)
    out = ehm({k: _t(v) for k, v in bp.items()}, {k: _t(v) for k, v in fp.items()})
    ref = lo.ehm_forward(body, flame, extra, bp, fp)
    for k in ("vertices", "joints", "joints_transform", "ver_transform_mat", "joint_transform_mat"):
        np.testing.assert_allclose(out[k].cpu().numpy(), ref[k], atol=ATOL, rtol=0, err_msg=k)


def test_ehm_broadcast_and_absent_params():
    """The coefficient-row packing (gsr_pack_rows): a one-row identity shape and head_scale broadcast
    over the frames, an absent global_pose (zero rows, EHM.py:94-96) -- against the oracle given the
    explicit equivalents."""
    from guava_renderer_amd import avatar, deform
    body, flame, extra = avatar.ehm_assets(seed=0)
    bp, fp = avatar.ehm_params(5, seed=3000)
    ehm = deform.EHMDeformer(body, flame, extra["smplx2flame_ind"], extra["l_eyelid"], extra["r_eyelid"],
                             device=DEV)
    gbp = {k: _t(v) for k, v in bp.items()}
    gbp["shape"] = _t(bp["shape"][:1])
    gbp["head_scale"] = _t(bp["head_scale"][0])
    del gbp["global_pose"]
    out = ehm(gbp, {k: _t(v) for k, v in fp.items()})
    rbp = dict(bp)
    rbp["head_scale"] = np.broadcast_to(bp["head_scale"][:1], bp["head_scale"].shape)
    rbp["global_pose"] = np.zeros_like(bp["global_pose"])
    ref = lo.ehm_forward(body, flame, extra, rbp, fp)
    for k in ("vertices", "joints", "ver_transform_mat"):
        np.testing.assert_allclose(out[k].cpu().numpy(), ref[k], atol=ATOL, rtol=0, err_msg=k)


def test_lbs_with_betas_b17_matrix_core_tails():
    """deform.lbs at B=17 (a partial 32-frame tile) on the SMPL-X-size model, vs the oracle."""
    from guava_renderer_amd import deform
    m, g, faces, betas, pose = _full_avatar(B=17, P=20000)
    verts, jt = deform.lbs(_t(betas), _t(pose), _t(m["v_template"]), _t(m["shapedirs"]), _t(m["posedirs"]),
                           _t(m["J_regressor"]), torch.from_numpy(m["parents"]), _t(m["lbs_weights"]))
    r_verts, r_jt, *_ = lo.lbs(betas, pose, m["v_template"], m["shapedirs"], m["posedirs"],
                               m["J_regressor"], m["parents"], m["lbs_weights"])
    np.testing.assert_allclose(verts.cpu().numpy(), r_verts, atol=ATOL, rtol=0)
    np.testing.assert_allclose(jt.cpu().numpy(), r_jt, atol=ATOL, rtol=0)


def test_config5_cross_reenactment_avatar_pipeline():
    """BASELINE config 5 as the bench runs it (`--config c5 --pipeline avatar`): 300k Gaussians (3 per
    UV texel), cross-reenactment inputs (target poses with the source identity, main/test.py:21-28,
    96-139), 1024x1024.  EHM + Gaussian assembly vs the oracle composition at full size (B=2), then
    frame 1 rendered through the batched entry, bit-exact with the CPU oracle on the same assets."""
    import oracle
    from guava_renderer_amd import avatar, scenes
    from guava_renderer_amd.pipeline import AvatarPipeline
    B, P, W = 2, 300000, 1024
    body, flame, extra = avatar.ehm_assets(seed=0)
    verts, faces, tex = avatar.template_mesh()
    g = avatar.gaussians(verts, faces, tex * 3, P=P, seed=0)
    tb, tf = avatar.ehm_params(B, seed=2000)
    sb, sf = avatar.ehm_params(1, seed=77)
    bp, fp = avatar.change_id_info(tb, tf, sb, sf)
    assert np.array_equal(bp["shape"][1], sb["shape"][0]) and np.array_equal(bp["body_pose"], tb["body_pose"])
    pipe = AvatarPipeline(body, flame, extra, g, B, W, W, R_capacity=30 * P * B, device=DEV)
    assert pipe.P == P
    cams = scenes.frame_cameras(B, W, W, seed=1000)
    views = _t(np.stack([c["viewmatrix"].reshape(16) for c in cams]))
    projs = _t(np.stack([c["projmatrix"].reshape(16) for c in cams]))
    tanf = _t(np.array([[c["tanfovx"], c["tanfovy"]] for c in cams], np.float32))
    col, inv, radii, d = pipe.render({k: _t(v) for k, v in bp.items()}, {k: _t(v) for k, v in fp.items()},
                                     views, projs, tanf)
    torch.cuda.synchronize()
    assert not pipe.rast.status()[1]
    # EHM vs the oracle composition (vertices / transforms at ATOL), then the Gaussian assembly from
    # the GPU's own deformed mesh (as test_full_smplx_lbs_and_gaussian_assembly): a face frame
    # amplifies the mesh's float32 error by 1 / edge length (~1e2 at SMPL-X's 1 cm edges), which is
    # the LBS's error, not the assembly's
    gbp, gfp = {k: _t(v) for k, v in bp.items()}, {k: _t(v) for k, v in fp.items()}
    ge = pipe.ehm(gbp, gfp)
    e = lo.ehm_forward(body, flame, extra, bp, fp)
    for k in ("vertices", "ver_transform_mat"):
        np.testing.assert_allclose(ge[k].cpu().numpy(), e[k], atol=ATOL, rtol=0, err_msg=k)
    gd = pipe.gauss(ge["vertices"], ge["ver_transform_mat"])
    for k in ("xyz", "rotation", "scaling"):  # the pipeline's deform is exactly these two calls
        assert torch.equal(gd[k], d[k]), k
    ref = lo.deform_gaussians(ge["vertices"].cpu().numpy(), ge["ver_transform_mat"].cpu().numpy(), extra["faces"],
                              g["vtx_rotations"], g["vtx_scales"], g["binding_face"], g["face_bary"],
                              g["local_xyz"], g["uv_rotations"], g["uv_scales"])
    np.testing.assert_allclose(d["xyz"].cpu().numpy(), ref["xyz"], atol=ATOL, rtol=0)
    np.testing.assert_allclose(d["scaling"].cpu().numpy(), ref["scaling"], atol=ATOL, rtol=0)
    q, rq = d["rotation"].cpu().numpy(), ref["rotation"]
    err = np.minimum(np.abs(q - rq).max(-1), np.abs(q + rq).max(-1))
    firm = ref["margin"] >= 1e-4
    assert firm.mean() > 0.99 and err[firm].max() < ATOL, err[firm].max()
    # the render of frame 1 from the GPU-deformed assets, bit-exact with the oracle
    oracle.set_threads(16)
    f = 1
    o_col, o_radii, o_inv, _ = oracle.forward(
        d["xyz"][f].cpu().numpy(), g["colors"], g["opacities"], d["scaling"][f].cpu().numpy(),
        d["rotation"][f].cpu().numpy(), None, cams[f]["viewmatrix"], cams[f]["projmatrix"], W, W,
        cams[f]["tanfovx"], cams[f]["tanfovy"], np.zeros(32, np.float32))
    np.testing.assert_array_equal(radii[f].cpu().numpy(), o_radii)
    np.testing.assert_array_equal(col[f].cpu().numpy(), o_col)
    np.testing.assert_array_equal(inv[f].cpu().numpy(), o_inv.reshape(W, W))
    # the fused forward (assembly inside the projection kernel, gsr_forward_batch_deformed): the
    # same images from the same EHM output, without materialising the deformed Gaussians
    c0, i0, r0 = col.clone(), inv.clone(), radii.clone()
    col2, inv2, radii2, d2 = pipe.render(gbp, gfp, views, projs, tanf, fused=True)
    torch.cuda.synchronize()
    assert d2 is None and not pipe.rast.status()[1]
    assert torch.equal(radii2, r0) and torch.equal(col2, c0) and torch.equal(inv2, i0)


def test_fused_deform_forward_equals_two_step_and_flags_bad_index():
    """gsr_forward_batch_deformed vs gsr_deform_gaussians + gsr_forward_batch on a small avatar
    (B=3, shared and per-frame cameras): identical images, invdepth and radii; an out-of-range
    binding face is flagged and its Gaussian dropped (NaN centre, radius 0) without a fault; a
    backward after the fused forward is refused."""
    from guava_renderer_amd import deform, scenes
    from guava_renderer_amd._lib import GsrError
    from guava_renderer_amd.batch import BatchRasterizer
    rng = np.random.default_rng(3)
    V, F, N, B, W = 400, 600, 1500, 3, 96
    faces = np.stack([rng.choice(V, 3, replace=False) for _ in range(F)]).astype(np.int32)
    bind = rng.integers(0, F, N).astype(np.int32)
    bind[17] = F + 3  # out of range

    def quats(n):
        q = rng.normal(size=(n, 4)).astype(np.float32)
        return q / np.linalg.norm(q, axis=1, keepdims=True)

    dfm = deform.GaussianDeformer(
        {"rotations": _t(quats(V)), "scales": _t(rng.uniform(0.005, 0.03, (V, 3)).astype(np.float32)),
         "opacities": _t(rng.uniform(0.2, 0.95, (V, 1)).astype(np.float32)),
         "colors": _t(rng.uniform(0, 1, (V, 32)).astype(np.float32))},
        {"rotations": _t(quats(N)), "scales": _t(rng.uniform(0.1, 1.5, (N, 3)).astype(np.float32)),
         "opacities": _t(rng.uniform(0.2, 0.95, (N, 1)).astype(np.float32)),
         "colors": _t(rng.uniform(0, 1, (N, 32)).astype(np.float32)),
         "local_pos": _t(rng.normal(scale=0.01, size=(N, 3)).astype(np.float32)), "binding_face": _t(bind),
         "face_bary": _t(rng.dirichlet(np.ones(3), N).astype(np.float32))}, _t(faces))
    verts = _t(rng.normal(scale=0.25, size=(B, V, 3)).astype(np.float32))
    T = np.broadcast_to(np.eye(4, dtype=np.float32), (B, V, 4, 4)).copy()
    T[..., :3, :3] += rng.normal(scale=0.1, size=(B, V, 3, 3)).astype(np.float32)
    T = _t(T)
    cams = scenes.frame_cameras(B, W, W, seed=5)
    views = _t(np.stack([c["viewmatrix"].reshape(16) for c in cams]))
    projs = _t(np.stack([c["projmatrix"].reshape(16) for c in cams]))
    tanf = _t(np.array([[c["tanfovx"], c["tanfovy"]] for c in cams], np.float32))
    bg = _t(rng.uniform(0, 1, (B, 32)).astype(np.float32))
    P = V + N
    rast = BatchRasterizer(B, P, W, W, R_capacity=64 * P * B, device=DEV)
    d = dfm(verts, T)
    col, inv, radii = rast.forward(d["xyz"], dfm.colors, dfm.opacity, d["scaling"], d["rotation"], views, projs,
                                   tanf, bg, forward_only=True)
    c0, i0, r0 = col.clone(), inv.clone(), radii.clone()
    assert dfm.bad_index()
    dfm.bad.zero_()
    col2, inv2, radii2 = rast.forward_deformed(dfm, verts, T, views, projs, tanf, bg)
    torch.cuda.synchronize()
    assert dfm.bad_index() and not rast.status()[1]
    assert (r0 > 0).sum() > P // 2 and r0[:, V + 17].eq(0).all()
    assert torch.equal(radii2, r0) and torch.equal(col2, c0) and torch.equal(inv2, i0)
    with pytest.raises(GsrError):
        rast.backward(d["xyz"], dfm.colors, dfm.opacity, d["scaling"], d["rotation"], views, projs, tanf, bg,
                      torch.ones_like(col2), torch.zeros_like(inv2))
