"""Camera matrices in the rasterizer's row-vector / transposed convention.

Restates /root/reference/utils/graphics_utils.py:15-50 (get_view_matrix, get_proj_matrix,
get_full_proj_matrix) and the canonical camera of dataset/data_loader.py:377-394, in numpy
float32 so tests, smoke and bench produce identical matrices on any host.
"""
import math

import numpy as np


def get_view_matrix(R, t):
    """graphics_utils.py:15-21: [R | t; 0 0 0 1]."""
    V = np.zeros((4, 4), np.float32)
    V[:3, :3] = R
    V[:3, 3] = np.asarray(t, np.float32).reshape(3)
    V[3, 3] = 1.0
    return V


def get_proj_matrix(tanfov, z_near=0.01, z_far=100.0):
    """graphics_utils.py:23-42 (z_sign = 1)."""
    tanfov = np.float32(tanfov)
    top = tanfov * np.float32(z_near)
    bottom = -top
    right = tanfov * np.float32(z_near)
    left = -right
    P = np.zeros((4, 4), np.float32)
    P[0, 0] = np.float32(2.0 * z_near) / (right - left)
    P[1, 1] = np.float32(2.0 * z_near) / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = 1.0
    P[2, 2] = np.float32(z_far / (z_far - z_near))
    P[2, 3] = np.float32(-(z_far * z_near) / (z_far - z_near))
    return P


def get_full_proj_matrix(w2c, tanfov):
    """graphics_utils.py:44-50: returns (viewmatrix, full_proj) both transposed (row-vector)."""
    w2c = np.asarray(w2c, np.float32)
    view = get_view_matrix(w2c[:3, :3], w2c[:3, 3]).T.copy()
    proj = get_proj_matrix(tanfov).T.copy()
    full = (view.astype(np.float32) @ proj.astype(np.float32)).astype(np.float32)
    return view, full


def look_at_w2c(yaw=0.0, pitch=0.0, distance=22.0, y_offset=0.6):
    """Canonical GUAVA camera (R=I, t=(0, 0.6, 22), data_loader.py:377-394) orbited by yaw/pitch
    around the avatar (the recipe of utils/camera_utils.py:72-88)."""
    cy, sy = math.cos(yaw), math.sin(yaw)
    cp, sp = math.cos(pitch), math.sin(pitch)
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]], np.float64)
    Rx = np.array([[1, 0, 0], [0, cp, -sp], [0, sp, cp]], np.float64)
    R = Rx @ Ry
    w2c = np.eye(4, dtype=np.float64)
    w2c[:3, :3] = R
    w2c[:3, 3] = [0.0, y_offset, distance]
    return w2c.astype(np.float32)


def camera(W, H, tanfov=1.0 / 24.0, yaw=0.0, pitch=0.0, distance=22.0):
    """All per-view raster settings fields as numpy values (GaussianRasterizationSettings, a1)."""
    w2c = look_at_w2c(yaw, pitch, distance)
    view, full = get_full_proj_matrix(w2c, tanfov)
    c2w = np.linalg.inv(w2c.astype(np.float64)).astype(np.float32)
    return dict(image_height=int(H), image_width=int(W), tanfovx=float(np.float32(tanfov)),
                tanfovy=float(np.float32(tanfov)), viewmatrix=view, projmatrix=full,
                campos=c2w[:3, 3].copy())
