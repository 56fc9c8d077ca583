"""Generates tests/golden/oracle_micro.npz: inputs and CPU-oracle outputs (forward state, image,
gradients) of two small scenes, pinned further by tests/test_oracle.py's float64 autograd check.
Re-run only when the numerics contract changes; the fixture is data, not code.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402
from helpers import make_scene  # noqa: E402


def scene_arrays(kind, P, W, H, seed):
    d = make_scene(kind, P, W, H, seed=seed)
    rng = np.random.default_rng(seed + 100)
    dL = rng.normal(size=(32, H, W)).astype(np.float32)
    dLinv = rng.normal(size=(1, H, W)).astype(np.float32)
    col, radii, invd, st = oracle.forward(d["means3D"], d["colors"], d["opacities"], d["scales"],
                                          d["rotations"], None, d["viewmatrix"], d["projmatrix"], W, H,
                                          d["tanfovx"], d["tanfovy"], d["bg"])
    g = oracle.backward(st, d["means3D"], d["colors"], d["opacities"], d["scales"], d["rotations"], None,
                        d["viewmatrix"], d["projmatrix"], W, H, d["tanfovx"], d["tanfovy"], d["bg"],
                        dL, dLinv)
    out = {}
    for k in ("means3D", "colors", "opacities", "scales", "rotations", "viewmatrix", "projmatrix",
              "campos", "bg"):
        out["in_" + k] = d[k]
    out["in_tan"] = np.array([d["tanfovx"], d["tanfovy"]], np.float32)
    out["in_size"] = np.array([W, H], np.int32)
    out["in_dL"] = dL
    out["in_dLinv"] = dLinv
    out["out_color"] = col
    out["out_invdepth"] = invd
    out["out_radii"] = radii
    for k in ("means2D", "depths", "conic_opacity", "tiles_touched", "point_list", "ranges",
              "final_T", "n_contrib"):
        out["st_" + k] = st[k]
    for name, v in zip(("means2D", "colors", "opacity", "means3D", "cov3D", "sh", "scales", "rotations"), g):
        out["grad_" + name] = v
    return out


def main():
    scenes = {"random": ("random", 300, 32, 32, 7), "avatar": ("avatar", 600, 32, 32, 8)}
    payload = {}
    for name, args in scenes.items():
        for k, v in scene_arrays(*args).items():
            payload[f"{name}__{k}"] = v
    path = os.path.join(HERE, "oracle_micro.npz")
    np.savez_compressed(path, **payload)
    print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
