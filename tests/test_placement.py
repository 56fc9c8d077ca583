"""Host logic of the render placement (include/gsr.h gsr_stream_create_cu_mask / gsr_set_render_stream,
guava_renderer_amd/parallel.py cu_masks): the prep and render CU masks partition the chip, and the
prep slice takes the same share of every XCD whether the mask's bit order interleaves the 8 XCDs
(CU i on XCD i mod 8) or runs through them in order (CU i on XCD i // 32)."""
import collections

import pytest

from guava_renderer_amd.parallel import cu_masks


@pytest.mark.parametrize("k", [8, 16, 32, 48, 64, 128])
def test_spread_slice_partitions_and_balances(k):
    prep, render = cu_masks(256, k, "spread")
    p = set()
    for wi, w in enumerate(prep):
        p |= {32 * wi + b for b in range(32) if (w >> b) & 1}
    r = set()
    for wi, w in enumerate(render):
        r |= {32 * wi + b for b in range(32) if (w >> b) & 1}
    assert len(p) == k and not (p & r) and (p | r) == set(range(256))
    assert set(collections.Counter(c % 8 for c in p).values()) == {k // 8}
    assert set(collections.Counter(c // 32 for c in p).values()) == {k // 8}


def test_lo_slice_and_no_split():
    prep, render = cu_masks(256, 40, "lo")
    assert prep[0] == 0xFFFFFFFF and prep[1] == 0xFF and all(w == 0 for w in prep[2:])
    assert render[1] == 0xFFFFFF00 and all(w == 0xFFFFFFFF for w in render[2:])
    full, full2 = cu_masks(256, 0)
    assert full == full2 == [0xFFFFFFFF] * 8
    with pytest.raises(ValueError):
        cu_masks(256, 256)


def test_rasterizer_module_state_is_an_nn_module():
    """GaussianRasterizer_32 builds nn.Module's state directly (one module per frame in GUAVA's loop,
    gaussian_render.py:37-51): the same attributes as nn.Module.__init__, fresh containers per
    instance, hooks / train / eval / state_dict behave as for any module."""
    import torch
    import torch.nn as nn
    from guava_renderer_amd.diff_gaussian_rasterization_32 import (GaussianRasterizationSettings,
                                                                   GaussianRasterizer_32)
    bg, v = torch.zeros(32), torch.eye(4)
    rs = GaussianRasterizationSettings(image_height=8, image_width=8, tanfovx=0.5, tanfovy=0.5, bg=bg,
                                       scale_modifier=1.0, viewmatrix=v, projmatrix=v, sh_degree=0, campos=bg[:3],
                                       prefiltered=False, debug=False, antialiasing=False)
    a, b = GaussianRasterizer_32(raster_settings=rs), GaussianRasterizer_32(rs)
    assert isinstance(a, nn.Module) and a.raster_settings is rs
    assert set(a.__dict__) - {"raster_settings"} == set(nn.Module().__dict__)
    assert a._parameters is not b._parameters and a._forward_pre_hooks is not b._forward_pre_hooks
    a.register_forward_pre_hook(lambda m, i: None)
    assert len(a._forward_pre_hooks) == 1 and len(b._forward_pre_hooks) == 0
    a.eval()
    assert not a.training and b.training and len(a.state_dict()) == 0
    with pytest.raises(Exception, match="one of either SHs or precomputed colors"):
        b(means3D=torch.zeros(1, 3), means2D=torch.zeros(1, 3), opacities=torch.ones(1, 1))
