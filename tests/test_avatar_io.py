"""On-disk avatar format (guava_renderer_amd/avatar_io.py): the canonical Gaussian PLY of
Ubody_Gaussian.save_gaussian_ply (models/UbodyAvatar/ubody_gaussian.py:350-373, :408-420).

No PLY ships with the reference and plyfile is not installed, so the layout is pinned by the
header text and record stride plyfile produces for that element, and by round trips; a file
written by the reference itself is "parity unpinned".  The GPU test renders a PLY-loaded avatar
through the batched entry and compares it bit-exactly with the oracle on the same attributes."""
import numpy as np
import pytest

from guava_renderer_amd import avatar_io, scenes


def _attrs(P=500, seed=0):
    d = scenes.random_cloud(P, seed)
    return d["means3D"], d["colors"][:, :3], d["opacities"], d["scales"], d["rotations"]


def test_header_and_stride(tmp_path):
    xyz, rgb, op, sc, rot = _attrs(37)
    p = tmp_path / "GS_canonical.ply"
    avatar_io.write_gaussian_ply(p, xyz, rgb, op, sc, rot)
    raw = p.read_bytes()
    hdr = (b"ply\nformat binary_little_endian 1.0\nelement vertex 37\n"
           + b"".join(b"property float %s\n" % n.encode() for n in avatar_io.PROPS) + b"end_header\n")
    assert raw.startswith(hdr)
    assert len(raw) == len(hdr) + 37 * 17 * 4  # 17 float32 properties per Gaussian
    rec = np.frombuffer(raw[len(hdr):], dtype="<f4").reshape(37, 17)
    np.testing.assert_array_equal(rec[:, 0:3], xyz)
    np.testing.assert_array_equal(rec[:, 3:6], 0.0)                        # normals
    np.testing.assert_allclose(rec[:, 6:9], rgb / avatar_io.SH_C0, rtol=1e-6)  # RGB -> SH DC
    np.testing.assert_allclose(rec[:, 9], np.log(op[:, 0] / (1 - op[:, 0])), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(rec[:, 10:13], np.log(sc), rtol=1e-6, atol=1e-6)
    np.testing.assert_array_equal(rec[:, 13:17], rot)


def test_round_trip_activation(tmp_path):
    xyz, rgb, op, sc, rot = _attrs(300, seed=4)
    p = tmp_path / "a.ply"
    avatar_io.write_gaussian_ply(p, xyz, rgb, op, sc, rot)
    a = avatar_io.activate(avatar_io.read_gaussian_ply(p))
    np.testing.assert_array_equal(a["means3D"], xyz)
    np.testing.assert_array_equal(a["rotations"], rot)
    np.testing.assert_allclose(a["opacities"], op, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(a["scales"], sc, rtol=1e-5)
    np.testing.assert_allclose(a["colors"][:, :3], rgb, rtol=1e-6, atol=1e-7)
    assert a["colors"].shape == (300, 32) and not a["colors"][:, 3:].any()


def test_reads_ascii_big_endian_and_extra_properties(tmp_path):
    xyz, rgb, op, sc, rot = _attrs(5, seed=2)
    p = tmp_path / "b.ply"
    avatar_io.write_gaussian_ply(p, xyz, rgb, op, sc, rot)
    ref = avatar_io.read_gaussian_ply(p)
    rec = np.frombuffer(p.read_bytes()[len(avatar_io.header(5)):], dtype="<f4").reshape(5, 17)
    # ascii, with a comment and an extra property the reader must skip over
    lines = ["ply", "format ascii 1.0", "comment written by a test", "element vertex 5"]
    lines += [f"property float {n}" for n in avatar_io.PROPS] + ["property float extra", "end_header"]
    lines += [" ".join(repr(float(v)) for v in list(r) + [7.0]) for r in rec]
    pa = tmp_path / "ascii.ply"
    pa.write_text("\n".join(lines) + "\n")
    got = avatar_io.read_gaussian_ply(pa)
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k])
    # big endian
    pb = tmp_path / "be.ply"
    pb.write_bytes(avatar_io.header(5).replace(b"binary_little_endian", b"binary_big_endian")
                   + rec.astype(">f4").tobytes())
    got = avatar_io.read_gaussian_ply(pb)
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k])


def test_rejects_malformed(tmp_path):
    p = tmp_path / "x.ply"
    p.write_bytes(b"not a ply\n")
    with pytest.raises(ValueError):
        avatar_io.read_gaussian_ply(p)
    p.write_bytes(b"ply\nformat binary_little_endian 1.0\nelement vertex 1\nproperty float x\nend_header\n" + b"\0" * 4)
    with pytest.raises(ValueError, match="lacks"):
        avatar_io.read_gaussian_ply(p)


@pytest.mark.gpu
def test_ply_avatar_renders_like_oracle(tmp_path):
    import torch

    from guava_renderer_amd import camera
    from guava_renderer_amd.batch import BatchRasterizer
    from helpers import oracle_forward

    d = scenes.avatar_cloud(6000, 1)
    p = tmp_path / "GS_canonical.ply"
    avatar_io.write_gaussian_ply(p, d["means3D"], d["colors"][:, :3], d["opacities"], d["scales"], d["rotations"])
    dev = torch.device("cuda")
    t = avatar_io.load_gaussian_ply(p, dev)
    W, H = 160, 128
    cam = camera.camera(W, H)
    host = avatar_io.activate(avatar_io.read_gaussian_ply(p))
    o = dict(host, **cam, bg=np.zeros(32, np.float32))
    o_col, o_radii, o_inv, _ = oracle_forward(o)
    rast = BatchRasterizer(1, 6000, W, H, R_capacity=64 * 6000, device=dev)
    view = torch.tensor(cam["viewmatrix"].reshape(1, 16), device=dev)
    proj = torch.tensor(cam["projmatrix"].reshape(1, 16), device=dev)
    tanf = torch.tensor([[cam["tanfovx"], cam["tanfovy"]]], dtype=torch.float32, device=dev)
    col, inv, radii = rast.forward(t["means3D"], t["colors"], t["opacities"], t["scales"], t["rotations"],
                                   view, proj, tanf, torch.zeros((1, 32), device=dev))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(radii[0].cpu().numpy(), o_radii)
    np.testing.assert_array_equal(col[0].cpu().numpy(), o_col)
    np.testing.assert_array_equal(inv[0].cpu().numpy().reshape(o_inv.shape), o_inv)
