"""Import shim: `from fused_ssim import fused_ssim` (as GUAVA's utils/loss_utils.py:7 does) resolves
to the MI355X implementation (guava_renderer_amd/fused_ssim.py)."""
from guava_renderer_amd.fused_ssim import (  # noqa: F401
    FusedSSIMMap, allowed_padding, fused_ssim, fusedssim, fusedssim_backward)
