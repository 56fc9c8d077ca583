"""The culling tests that decide which (Gaussian, pixel rectangle) pairs the GPU never blends
(csrc/gsr_cull.h): built for the host with hipcc and run on random conics near the origin and at
large pixel coordinates (tools/quad_mask_check.cpp, tools/strip_mask_check.cpp).  The single-frame
quad masks binning stores (quad_reach4, k_quad_masks) must equal box_reach on each quad and never clear
a quad holding a pixel centre at alpha >= 1/255 (float64 brute force), so the quad render waves' lists
stay decision-preserving; the conservative reach boxes (A/B only) must never clear one either; and the
scatter's strip masks (sub_reach4<8>) must equal the four box_reach calls and never clear a strip
holding such a pixel."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_quad_masks_match_box_reach_and_never_drop(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    exe = tmp_path / "qmc"
    subprocess.run([hipcc, "-O2", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "-I",
                    os.path.join(ROOT, "guava_renderer_amd", "csrc"), os.path.join(ROOT, "tools", "quad_mask_check.cpp"),
                    "-o", str(exe)], check=True, capture_output=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    print(out.stdout)
    assert out.returncode == 0, out.stdout
    assert "mismatches vs box_reach 0, missed 0" in out.stdout
    assert "reach boxes: missed 0," in out.stdout


def test_strip_masks_match_box_reach_loop_and_never_drop(tmp_path):
    """binning's strip_mask (sub_reach4<8>: the tile's four strips with shared terms) gives the same
    bits as the four box_reach calls, and never clears a strip holding a pixel centre at alpha >= 1/255
    (float64 brute force, tools/strip_mask_check.cpp)."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    exe = tmp_path / "smc"
    subprocess.run([hipcc, "-O2", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "-I",
                    os.path.join(ROOT, "guava_renderer_amd", "csrc"), "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tools", "strip_mask_check.cpp"), "-o", str(exe)], check=True, capture_output=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    print(out.stdout)
    assert out.returncode == 0, out.stdout
    assert "wrongly cleared 0, mismatches vs the box_reach loop 0" in out.stdout
