#
# The Python/autograd surface below follows diff_gaussian_rasterization_32/__init__.py of the
# reference, which carries this notice:
#
# Copyright (C) 2023, Inria
# GRAPHDECO research group, https://team.inria.fr/graphdeco
# All rights reserved.
#
# This software is free for non-commercial, research and evaluation use
# under the terms of the LICENSE.md file.
#
# For inquiries contact  george.drettakis@inria.fr
#
# (LICENSE.md: /root/reference/submodules/diff-gaussian-rasterization-32/LICENSE.md, reproduced in
# this package as LICENSE.md.)
"""Drop-in replacement of diff_gaussian_rasterization_32 for AMD MI355X (gfx950).

Python/autograd surface identical to the reference package
(/root/reference/submodules/diff-gaussian-rasterization-32/diff_gaussian_rasterization_32/
__init__.py): `rasterize_gaussians` (:21-42), `_RasterizeGaussians` (:44-141),
`GaussianRasterizationSettings` (:143-156) and `GaussianRasterizer_32` (:158-207), so
models/UbodyAvatar/gaussian_render.py, render_motion.py and main/test.py run unchanged.
The native `_C` module is backed by the HIP kernels of libgsr.so; there is no CPU path.
"""
import os
from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

# GSR_INFERENCE_PATH=0: inference calls take the autograd Function too (A/B of _C.rasterize_inference)
_INFERENCE_PATH = os.environ.get("GSR_INFERENCE_PATH", "1") != "0"
_EMPTY = torch.Tensor([])


def cpu_deep_copy_tuple(input_tuple):
    copied_tensors = [item.cpu().clone() if isinstance(item, torch.Tensor) else item for item in input_tuple]
    return tuple(copied_tensors)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                        cov3Ds_precomp, raster_settings):
    # whether autograd will keep this call's scratch buffers for backward (known only here: the
    # Function's forward runs with grad mode off): then the binning buffer is sized to the exact
    # instance count (the reference's host read-back of num_rendered), otherwise the forward runs
    # without a host synchronisation and its transient buffer is released with the call
    inputs = (means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp)
    record = torch.is_grad_enabled() and any(isinstance(t, torch.Tensor) and t.requires_grad for t in inputs)
    if (_INFERENCE_PATH and not record and not raster_settings.debug and not raster_settings.prefiltered
            and (sh is None or sh.numel() == 0)):
        # nothing will call backward: the same images without the autograd node and the per-call
        # scratch allocations (_C.rasterize_inference; None when it does not apply)
        out = _C.rasterize_inference(raster_settings.bg, means3D, colors_precomp, opacities, scales, rotations,
                                     raster_settings.scale_modifier, cov3Ds_precomp, raster_settings.viewmatrix,
                                     raster_settings.projmatrix, raster_settings.tanfovx, raster_settings.tanfovy,
                                     raster_settings.image_height, raster_settings.image_width,
                                     raster_settings.antialiasing)
        if out is not None:
            return out
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales,
                                     rotations, cov3Ds_precomp, raster_settings, record)


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                cov3Ds_precomp, raster_settings, _for_backward=True):
        # argument order of the native call (reference __init__.py:60-81)
        args = (
            raster_settings.bg,
            means3D,
            colors_precomp,
            opacities,
            scales,
            rotations,
            raster_settings.scale_modifier,
            cov3Ds_precomp,
            raster_settings.viewmatrix,
            raster_settings.projmatrix,
            raster_settings.tanfovx,
            raster_settings.tanfovy,
            raster_settings.image_height,
            raster_settings.image_width,
            sh,
            raster_settings.sh_degree,
            raster_settings.campos,
            raster_settings.prefiltered,
            raster_settings.antialiasing,
            raster_settings.debug,
        )
        num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer, invdepths = \
            _C.rasterize_gaussians(*args, exact_binning=bool(_for_backward))
        ctx.raster_settings = raster_settings
        ctx.num_rendered = num_rendered
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh,
                              opacities, geomBuffer, binningBuffer, imgBuffer)
        return color, radii, invdepths

    @staticmethod
    def backward(ctx, grad_out_color, _, grad_out_depth):
        num_rendered = ctx.num_rendered
        raster_settings = ctx.raster_settings
        (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, opacities,
         geomBuffer, binningBuffer, imgBuffer) = ctx.saved_tensors
        args = (raster_settings.bg,
                means3D,
                radii,
                colors_precomp,
                opacities,
                scales,
                rotations,
                raster_settings.scale_modifier,
                cov3Ds_precomp,
                raster_settings.viewmatrix,
                raster_settings.projmatrix,
                raster_settings.tanfovx,
                raster_settings.tanfovy,
                grad_out_color,
                grad_out_depth,
                sh,
                raster_settings.sh_degree,
                raster_settings.campos,
                geomBuffer,
                num_rendered,
                binningBuffer,
                imgBuffer,
                raster_settings.antialiasing,
                raster_settings.debug)
        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp,
         grad_sh, grad_scales, grad_rotations) = _C.rasterize_gaussians_backward(*args)
        grads = (
            grad_means3D,
            grad_means2D,
            grad_sh,
            grad_colors_precomp,
            grad_opacities,
            grad_scales,
            grad_rotations,
            grad_cov3Ds_precomp,
            None,
            None,
        )
        return grads


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool
    antialiasing: bool


def _module_state_factory():
    """nn.Module.__init__'s instance attributes, as a function returning fresh containers: GUAVA builds
    one GaussianRasterizer_32 per frame (gaussian_render.py:37-51), and nn.Module.__init__ (API-usage
    logging, ~17 attribute sets through Module.__setattr__ paths) is a sizeable share of the
    per-frame host time on the serial drop-in loop.  The attributes and their types are taken from a
    real nn.Module of this torch version, so the instance is an ordinary nn.Module."""
    proto = nn.Module().__dict__
    scalars = {k: v for k, v in proto.items() if not isinstance(v, (dict, set, list))}
    containers = [(k, type(v)) for k, v in proto.items() if isinstance(v, (dict, set, list))]

    def fresh():
        d = dict(scalars)
        for k, ty in containers:
            d[k] = ty()
        return d
    return fresh


_module_state = _module_state_factory()


class GaussianRasterizer_32(nn.Module):
    def __init__(self, raster_settings):
        # (nn.Module.__init__'s state, built directly: _module_state_factory)
        d = self.__dict__
        d.update(_module_state())
        d["raster_settings"] = raster_settings

    def markVisible(self, positions):
        # Mark visible points (based on frustum culling for camera) with a boolean
        with torch.no_grad():
            raster_settings = self.raster_settings
            visible = _C.mark_visible(positions, raster_settings.viewmatrix,
                                      raster_settings.projmatrix)
        return visible

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None,
                rotations=None, cov3D_precomp=None):
        raster_settings = self.raster_settings

        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')

        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')

        # (one shared empty CPU float tensor, as the reference's torch.Tensor([]): only read, never
        # written, and not built again on every call of the per-frame loop)
        if shs is None:
            shs = _EMPTY
        if colors_precomp is None:
            colors_precomp = _EMPTY
        if scales is None:
            scales = _EMPTY
        if rotations is None:
            rotations = _EMPTY
        if cov3D_precomp is None:
            cov3D_precomp = _EMPTY

        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales,
                                   rotations, cov3D_precomp, raster_settings)


__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer_32", "rasterize_gaussians"]
