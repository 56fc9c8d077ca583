"""Synthetic inputs for BASELINE.json's configs, as numpy float32 arrays.

Value distributions mirror GUAVA's decoders/deformer:
  opacity  sigmoid(N(0,1.5)), pruned at <= 0.001      feature_decoder.py:52,123; config.yaml:17
  scale    0.05*sigmoid(N(0,1)) (vertex Gaussians)     feature_decoder.py:55
           exp(N(-0.7,0.3)) * face scale (UV Gaussians) feature_decoder.py:126; ubody_gaussian.py:271
  rotation normalize(N(0,1)^4), wxyz                   feature_decoder.py:58,129
  features ch0-2 U(0,1) (sigmoid'd RGB), ch3-31 N(0,1) ubody_gaussian.py:186-187
  bg       zeros[32]                                   gaussian_render.py:35
"""
import os

import numpy as np

C = 32
_FIXTURE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests",
                        "golden", "avatar_template.npz")


def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def _attributes(rng, P, scale):
    op = _sigmoid(rng.normal(0.0, 1.5, P)).astype(np.float32)
    op = np.maximum(op, np.float32(0.0011))  # GUAVA prunes opacity <= 0.001 (config.yaml:17)
    q = rng.normal(size=(P, 4)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    feats = np.empty((P, C), np.float32)
    feats[:, :3] = rng.uniform(0.0, 1.0, (P, 3))
    feats[:, 3:] = rng.normal(size=(P, C - 3))
    return dict(opacities=op.reshape(P, 1), rotations=q.astype(np.float32),
                scales=scale.astype(np.float32), colors=feats)


def random_cloud(P=10000, seed=0):
    """Config 1: P random Gaussians near the canonical camera's look-at point."""
    rng = np.random.default_rng(seed)
    means = np.empty((P, 3), np.float32)
    means[:, 0] = rng.uniform(-0.8, 0.8, P)
    means[:, 1] = rng.uniform(-0.8, 0.8, P) - 0.6
    means[:, 2] = rng.uniform(-0.3, 0.3, P)
    scale = 0.05 * _sigmoid(rng.normal(size=(P, 3)))
    d = _attributes(rng, P, scale)
    d["means3D"] = means
    return d


def _face_frames(verts, faces):
    """compute_face_orientation (utils/graphics_utils.py:61-80), return_scale=True, numpy."""
    v0, v1, v2 = verts[faces[:, 0]], verts[faces[:, 1]], verts[faces[:, 2]]

    def nrm(x):
        return x / np.sqrt(np.maximum((x * x).sum(-1, keepdims=True), 1e-20))
    a0 = nrm(v1 - v0)
    a1 = nrm(np.cross(a0, v2 - v0))
    a2 = -nrm(np.cross(a1, a0))
    s0 = np.sqrt(np.maximum(((v1 - v0) ** 2).sum(-1, keepdims=True), 1e-20))
    s1 = np.abs((a2 * (v2 - v0)).sum(-1, keepdims=True))
    return np.stack([a0, a1, a2], -1), ((s0 + s1) / 2)[:, 0]


def avatar_cloud(P=100000, seed=0, gaussians_per_texel=1):
    """Config 2/3/5: SMPL-X template vertex Gaussians + one Gaussian per covered UV texel bound to
    its face at a random barycentric point, pruned at random to P.  The template is
    rotated to face the canonical camera (head up in the image)."""
    rng = np.random.default_rng(seed)
    fx = np.load(_FIXTURE)
    verts = fx["verts"].astype(np.float32)
    faces = fx["faces"].astype(np.int64)
    cnt = fx["texel_count"].astype(np.int64) * int(gaussians_per_texel)
    # place: rotate 180 deg about x (faces the camera, head up), feet below the frame
    verts = np.stack([verts[:, 0], -verts[:, 1] - 0.85, -verts[:, 2]], 1).astype(np.float32)
    _, fscale = _face_frames(verts, faces)
    face_of = np.repeat(np.arange(faces.shape[0]), cnt)
    N = face_of.shape[0]
    bary = rng.dirichlet([1.0, 1.0, 1.0], N).astype(np.float32)
    tri = verts[faces[face_of]]  # N,3,3
    uv_xyz = np.einsum("nk,nkj->nj", bary, tri).astype(np.float32)
    # small normal offset (GUAVA's local_xyz) so UV Gaussians do not all lie on the surface
    uv_xyz += rng.normal(0.0, 0.002, (N, 3)).astype(np.float32)
    uv_scale = np.exp(rng.normal(-0.7, 0.3, (N, 3))) * fscale[face_of][:, None]
    v_scale = 0.05 * _sigmoid(rng.normal(size=(verts.shape[0], 3)))
    means = np.concatenate([verts, uv_xyz], 0)
    scale = np.concatenate([v_scale, uv_scale], 0)
    total = means.shape[0]
    if P < total:
        keep = np.sort(rng.choice(total, P, replace=False))
    else:
        keep = np.arange(total)
    means = means[keep]
    scale = scale[keep]
    d = _attributes(rng, means.shape[0], scale)
    d["means3D"] = np.ascontiguousarray(means, np.float32)
    return d


def frame_cameras(n, W, H, seed=1000):
    """n distinct cameras around the avatar (yaw +-0.35, pitch +-0.3: config 3)."""
    from .camera import camera
    rng = np.random.default_rng(seed)
    cams = []
    for i in range(n):
        if i == 0:
            yaw, pitch = 0.0, 0.0
        else:
            yaw, pitch = rng.uniform(-0.35, 0.35), rng.uniform(-0.3, 0.3)
        cams.append(camera(W, H, yaw=yaw, pitch=pitch))
    return cams
