"""On-disk avatar format: the canonical Gaussian PLY GUAVA writes.

`Ubody_Gaussian.save_gaussian_ply(save_path)` (models/UbodyAvatar/ubody_gaussian.py:350-373, attribute
list :408-420) stores the canonical avatar -- vertex Gaussians first, then UV Gaussians -- as one
binary little-endian PLY element `vertex` of float32 properties

    x y z nx ny nz f_dc_0 f_dc_1 f_dc_2 opacity scale_0 scale_1 scale_2 rot_0 rot_1 rot_2 rot_3

with the stored (pre-activation) values
    f_dc     = rgb / 0.28209479177387814        (RGB -> SH DC, :355)
    opacity  = inverse_sigmoid(opacity)         (:356-357)
    scale_k  = log(scaling_k)                   (:358-359)
    rot      = the wxyz quaternion as held      (:360)
    normals  = 0                                (:362)

and `plyfile.PlyData([el]).write` (text=False, native byte order) frames it with the standard
header.  This module reads and writes exactly that layout with numpy (plyfile is not a dependency)
and uploads it into the rasterizer's input layout: `load_gaussian_ply(...)` ->
`to_device(...)` gives means3D [P,3], opacities [P,1] (sigmoid), scales [P,3] (exp),
rotations [P,4] and colors [P,32] (RGB in channels 0-2; the PLY carries no other channels, so
channels 3-31 are zero -- GUAVA's 32-channel features live only in the decoder's output).

The reference's other avatar file, the `torch.save`d `Ubody_Gaussian` module of create_avatar.py:64-70,
is a pickle of a whole module and is deliberately not loaded (unpickling executes code).

Parity: no PLY ships with the reference and plyfile is not installed here, so the byte layout is
pinned by the header/stride checks and round trips in tests/test_avatar_io.py ("parity unpinned"
against a file written by the reference itself).
"""
import io

import numpy as np

SH_C0 = 0.28209479177387814
PROPS = ("x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2", "opacity",
         "scale_0", "scale_1", "scale_2", "rot_0", "rot_1", "rot_2", "rot_3")
C = 32

_PLY_TYPES = {"float": "f4", "float32": "f4", "double": "f8", "float64": "f8", "uchar": "u1",
              "uint8": "u1", "char": "i1", "int8": "i1", "ushort": "u2", "uint16": "u2",
              "short": "i2", "int16": "i2", "uint": "u4", "uint32": "u4", "int": "i4", "int32": "i4"}


def _inverse_sigmoid(x):
    x = np.asarray(x, np.float64)
    return np.log(x / (1.0 - x))


def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-np.asarray(x, np.float64)))


def header(n):
    """The header plyfile writes for save_gaussian_ply's element (binary, little endian)."""
    lines = ["ply", "format binary_little_endian 1.0", f"element vertex {int(n)}"]
    lines += [f"property float {p}" for p in PROPS]
    lines.append("end_header")
    return ("\n".join(lines) + "\n").encode("ascii")


def write_gaussian_ply(path, xyz, rgb, opacity, scaling, rotation):
    """save_gaussian_ply's file from activated attributes: xyz [P,3], rgb [P,3] (the first three
    feature channels), opacity [P] or [P,1] in (0,1), scaling [P,3] > 0, rotation [P,4] wxyz."""
    xyz = np.asarray(xyz, np.float32).reshape(-1, 3)
    n = xyz.shape[0]
    rec = np.zeros(n, dtype=[(p, "<f4") for p in PROPS])
    rec["x"], rec["y"], rec["z"] = xyz[:, 0], xyz[:, 1], xyz[:, 2]
    f_dc = (np.asarray(rgb, np.float32).reshape(n, 3) / np.float32(SH_C0)).astype(np.float32)
    for k in range(3):
        rec[f"f_dc_{k}"] = f_dc[:, k]
    rec["opacity"] = _inverse_sigmoid(np.asarray(opacity, np.float64).reshape(n)).astype(np.float32)
    sc = np.log(np.asarray(scaling, np.float64).reshape(n, 3)).astype(np.float32)
    rot = np.asarray(rotation, np.float32).reshape(n, 4)
    for k in range(3):
        rec[f"scale_{k}"] = sc[:, k]
    for k in range(4):
        rec[f"rot_{k}"] = rot[:, k]
    with open(path, "wb") as f:
        f.write(header(n))
        f.write(rec.tobytes())


def _parse_header(f):
    first = f.readline()
    if first.strip() != b"ply":
        raise ValueError("not a PLY file")
    fmt, n, props, in_vertex = None, None, [], False
    while True:
        line = f.readline()
        if not line:
            raise ValueError("PLY header has no end_header")
        tok = line.decode("ascii", "replace").split()
        if not tok or tok[0] in ("comment", "obj_info"):
            continue
        if tok[0] == "end_header":
            break
        if tok[0] == "format":
            fmt = tok[1]
        elif tok[0] == "element":
            in_vertex = tok[1] == "vertex"
            if in_vertex:
                n = int(tok[2])
            elif n is None:
                raise ValueError(f"PLY element {tok[1]!r} before 'vertex' is not supported")
        elif tok[0] == "property" and in_vertex:
            if tok[1] == "list":
                raise ValueError("list properties are not supported in the Gaussian element")
            if tok[1] not in _PLY_TYPES:
                raise ValueError(f"unknown PLY property type {tok[1]!r}")
            props.append((tok[2], _PLY_TYPES[tok[1]]))
    if n is None:
        raise ValueError("PLY has no vertex element")
    return fmt, n, props


def read_gaussian_ply(path):
    """Reads save_gaussian_ply's file -> dict of the stored (pre-activation) float32 arrays:
    xyz [P,3], f_dc [P,3], opacity [P,1], scale [P,3], rotation [P,4]."""
    with open(path, "rb") as f:
        fmt, n, props = _parse_header(f)
        if fmt == "binary_little_endian":
            dt = np.dtype([(name, "<" + t) for name, t in props])
            rec = np.frombuffer(f.read(n * dt.itemsize), dtype=dt, count=n)
        elif fmt == "binary_big_endian":
            dt = np.dtype([(name, ">" + t) for name, t in props])
            rec = np.frombuffer(f.read(n * dt.itemsize), dtype=dt, count=n)
        elif fmt == "ascii":
            vals = np.loadtxt(io.StringIO(f.read().decode("ascii")), dtype=np.float64, max_rows=n, ndmin=2)
            rec = {name: vals[:, i] for i, (name, _) in enumerate(props)}
        else:
            raise ValueError(f"unsupported PLY format {fmt!r}")
    names = {p for p, _ in props}
    missing = [p for p in PROPS if p not in names and not p.startswith("n")]
    if missing:
        raise ValueError(f"PLY lacks Gaussian properties {missing}")

    def cols(*ks):
        return np.stack([np.asarray(rec[k], np.float32) for k in ks], axis=1)

    return {"xyz": cols("x", "y", "z"), "f_dc": cols("f_dc_0", "f_dc_1", "f_dc_2"),
            "opacity": cols("opacity"), "scale": cols("scale_0", "scale_1", "scale_2"),
            "rotation": cols("rot_0", "rot_1", "rot_2", "rot_3")}


def activate(stored):
    """Stored PLY values -> the rasterizer's inputs (numpy float32): means3D, opacities (sigmoid),
    scales (exp), rotations (as stored, wxyz; the rasterizer does not normalise, forward.cu:123)
    and colors [P,32] = (f_dc * SH_C0, 0...)."""
    n = stored["xyz"].shape[0]
    colors = np.zeros((n, C), np.float32)
    colors[:, :3] = stored["f_dc"] * np.float32(SH_C0)
    return {"means3D": np.ascontiguousarray(stored["xyz"], np.float32),
            "opacities": _sigmoid(stored["opacity"]).astype(np.float32),
            "scales": np.exp(stored["scale"].astype(np.float64)).astype(np.float32),
            "rotations": np.ascontiguousarray(stored["rotation"], np.float32),
            "colors": colors}


def to_device(attrs, device="cuda"):
    """Activated attributes -> contiguous torch tensors on `device` (one host-to-device copy each)."""
    import torch
    dev = torch.device(device)
    return {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in attrs.items()}


def load_gaussian_ply(path, device="cuda"):
    """read_gaussian_ply -> activate -> to_device."""
    return to_device(activate(read_gaussian_ply(path)), device)
