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
