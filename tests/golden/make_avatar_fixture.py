"""Builds tests/golden/avatar_template.npz from the reference's shipped SMPL-X assets.

Run ONLY in the build container (reads /root/reference); the GPU box uses the committed npz.
Data taken (no code): template vertices of assets/SMPLX/smplx_uv.obj, faces of
assets/SMPLX/smplx_faces.npy, and the per-face texel count of
assets/SMPLX/uv_masks/uv_mask512_with_faceid_smplx.npy (the UV-texel Gaussians GUAVA binds to
faces, ubody_gaussian.py:260-271).  Used by guava_renderer_amd/scenes.py to build the
BASELINE config-2 "pretrained-avatar-like" synthetic cloud, plus the SMPL-X -> FLAME
vertex map and the FLAME eyelid blend shapes (assets/SMPLX/SMPL-X__FLAME_vertex_ids.npy,
flame_{l,r}_eyelid.npy) used by the EHM head splice (guava_renderer_amd/avatar.py).
"""
import os
import numpy as np

REF = "/root/reference/assets/SMPLX"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "avatar_template.npz")

verts = []
with open(os.path.join(REF, "smplx_uv.obj")) as fh:
    for line in fh:
        if line.startswith("v "):
            verts.append([float(x) for x in line.split()[1:4]])
verts = np.asarray(verts, np.float32)
faces = np.load(os.path.join(REF, "smplx_faces.npy")).astype(np.uint16)
mask = np.load(os.path.join(REF, "uv_masks", "uv_mask512_with_faceid_smplx.npy"))
counts = np.bincount(mask[mask >= 0], minlength=faces.shape[0]).astype(np.uint16)
# EHM's FLAME-head mapping and eyelid blend shapes (SMPLX.py:191-193; used by EHM.py:72-74,122-124)
smplx2flame = np.load(os.path.join(REF, "SMPL-X__FLAME_vertex_ids.npy")).astype(np.uint16)
l_eyelid = np.load(os.path.join(REF, "flame_l_eyelid.npy")).astype(np.float32)
r_eyelid = np.load(os.path.join(REF, "flame_r_eyelid.npy")).astype(np.float32)
np.savez_compressed(OUT, verts=verts, faces=faces, texel_count=counts, smplx2flame_ind=smplx2flame,
                    l_eyelid=l_eyelid, r_eyelid=r_eyelid)
print(OUT, verts.shape, faces.shape, int(counts.sum()), int((counts > 0).sum()))
