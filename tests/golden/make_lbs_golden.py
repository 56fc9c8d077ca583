"""Builds tests/golden/lbs_golden.npz: outputs of the REFERENCE's own LBS code on synthetic inputs.

Run ONLY in the build container (imports /root/reference/models/modules/flame/lbs.py by file
path; the GPU box only sees the committed npz):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_lbs_golden.py

Inputs are regenerated deterministically by tests/golden/lbs_cases.py (seeded numpy); the npz keeps
the reference outputs plus a SHA-256 of every input array, so a drifting generator is detected
instead of silently comparing against stale vectors.
"""
import importlib.util
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import lbs_cases  # noqa: E402

REF = "/root/reference/models/modules/flame/lbs.py"
OUT = os.path.join(HERE, "lbs_golden.npz")
OUT_FULL = os.path.join(HERE, "lbs_golden_full.npz")  # SMPL-X / FLAME full-size cases


def _ref_module():
    spec = importlib.util.spec_from_file_location("ref_flame_lbs", REF)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def run_cases(ref, cases):
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x))  # noqa: E731
    out = {}
    for name, c in cases.items():
        out[f"{name}/sha"] = np.frombuffer(lbs_cases.digest(c).encode(), np.uint8)
        if c["kind"] == "rodrigues":
            out[f"{name}/rot"] = ref.batch_rodrigues(t(c["rot_vecs"])).numpy()
            continue
        par = torch.from_numpy(c["parents"].astype(np.int64))
        joff = t(c["joints_offset"]) if c.get("joints_offset") is not None else None
        if c["kind"] == "lbs":
            verts, jt = ref.lbs(t(c["betas"]), t(c["pose"]), t(c["v_template"])[None].expand(c["B"], -1, -1),
                                t(c["shapedirs"]), t(c["posedirs"]), t(c["J_regressor"]), par,
                                t(c["lbs_weights"]), joints_offset=joff)
            out[f"{name}/verts"] = verts.numpy()
            out[f"{name}/J_transformed"] = jt.numpy()
        else:  # lbs_wobeta
            verts, jt, J, T, A = ref.lbs_wobeta(t(c["pose"]), t(c["v_shaped"]), t(c["posedirs"]),
                                                t(c["J_regressor"]), par, t(c["lbs_weights"]),
                                                joints_offset=joff, pose2rot=c["pose2rot"])
            out[f"{name}/verts"] = verts.numpy()
            out[f"{name}/J_transformed"] = jt.numpy()
            out[f"{name}/J"] = J.numpy()
            out[f"{name}/T"] = T.numpy()
            out[f"{name}/A"] = A.numpy()
    return out


def main():
    ref = _ref_module()
    for path, cases in ((OUT, lbs_cases.all_cases()), (OUT_FULL, lbs_cases.full_cases())):
        out = run_cases(ref, cases)
        np.savez_compressed(path, **out)
        print(path, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
