"""Import shim: `from diff_gaussian_rasterization_32 import ...` (as GUAVA's
models/UbodyAvatar/gaussian_render.py:4 does) resolves to the MI355X implementation."""
from guava_renderer_amd.diff_gaussian_rasterization_32 import *  # noqa: F401,F403
from guava_renderer_amd.diff_gaussian_rasterization_32 import (  # noqa: F401
    GaussianRasterizationSettings, GaussianRasterizer_32, _C, _RasterizeGaussians,
    cpu_deep_copy_tuple, rasterize_gaussians)
