"""Per-frame avatar animation path of GUAVA on one GPU: deform -> rasterize, B frames per call.

The reference runs, per frame of main/test.py:70-76 (and render_motion.py:302-306):
    deformed = Ubody_Gaussian.forward(target)      ubody_gaussian.py:245-289  (EHM.forward inside)
    render   = GaussianRenderer.forward(deformed)  gaussian_render.py:19-67    (one rasterizer call
                                                                              per frame)
AvatarPipeline does the same work for B frames with one launch per stage and no host
synchronisation: EHMDeformer (FLAME head + SMPL-X body LBS), GaussianDeformer (vertex + UV
Gaussians), BatchRasterizer (preprocess, binning, depth order, 32-channel compositing).
"""
import numpy as np
import torch

from .batch import BatchRasterizer
from .deform import EHMDeformer, GaussianDeformer

C = 32


class AvatarPipeline:
    def __init__(self, body, flame, extra, gaussians, B, W, H, R_capacity=None, device="cuda"):
        dev = torch.device(device)
        t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)  # noqa: E731
        self.dev = dev
        self.ehm = EHMDeformer(body, flame, extra["smplx2flame_ind"], extra["l_eyelid"],
                               extra["r_eyelid"], device=dev)
        g = gaussians
        V = body["v_template"].shape[0]
        self.gauss = GaussianDeformer(
            {"rotations": t(g["vtx_rotations"]), "scales": t(g["vtx_scales"]),
             "opacities": t(g["opacities"][:V]), "colors": t(g["colors"][:V])},
            {"rotations": t(g["uv_rotations"]), "scales": t(g["uv_scales"]),
             "opacities": t(g["opacities"][V:]), "colors": t(g["colors"][V:]),
             "local_pos": t(g["local_xyz"]), "binding_face": t(g["binding_face"]),
             "face_bary": t(g["face_bary"])}, t(extra["faces"]), apply_rgb_sigmoid=False)
        self.P = self.gauss.V + self.gauss.N
        self.B, self.W, self.H = B, W, H
        self.rast = BatchRasterizer(B, self.P, W, H, R_capacity=R_capacity, device=dev)
        self.bg = torch.zeros((B, C), dtype=torch.float32, device=dev)

    def deform(self, body_params, flame_params):
        e = self.ehm(body_params, flame_params)
        return self.gauss(e["vertices"], e["ver_transform_mat"])

    def render(self, body_params, flame_params, views, projs, tanfov, refine=None, fused=False):
        """views / projs [B,16] (graphics_utils.py:44-50 layout), tanfov [B,2] ->
        (color [B,32,H,W], invdepth [B,H,W], radii [B,P], deformed assets).  refine: optional
        batch.RefineHead (the refiner's first conv fused into the render; output in refine.out).
        fused: the Gaussian assembly runs inside the projection kernel (gsr_forward_batch_deformed);
        the images are the same, the deformed assets are not materialised (returned as None)."""
        if fused:
            if refine is not None:
                raise ValueError("fused=True has no refiner epilogue; pass fused=False with refine")
            e = self.ehm(body_params, flame_params)
            col, inv, radii = self.rast.forward_deformed(self.gauss, e["vertices"], e["ver_transform_mat"], views,
                                                         projs, tanfov, self.bg)
            return col, inv, radii, None
        d = self.deform(body_params, flame_params)
        col, inv, radii = self.rast.forward(d["xyz"], self.gauss.colors, self.gauss.opacity,
                                            d["scaling"], d["rotation"], views, projs, tanfov, self.bg,
                                            refine=refine, forward_only=True)
        return col, inv, radii, d
