"""Run the bench's avatar deformation (EHM LBS + Gaussian assembly, 32 frames, P = 100k) alone,
for counter passes and kernel traces of the deform kernels:  python tools/deform_only.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from guava_renderer_amd import avatar
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda:0")
    t = lambda x: torch.as_tensor(x, device=dev)  # noqa: E731
    B, P = 32, 100000
    body, flame, extra = avatar.ehm_assets(seed=0)
    verts, faces, tex = avatar.template_mesh()
    g = avatar.gaussians(verts, faces, tex, P=P, seed=0)
    bp, fp = avatar.ehm_params(B, seed=1000)
    from guava_renderer_amd.pipeline import AvatarPipeline
    pipe = AvatarPipeline(body, flame, extra, g, B, 512, 512, R_capacity=1 << 20, device=dev)
    bpt = {k: t(v) for k, v in bp.items()}
    fpt = {k: t(v) for k, v in fp.items()}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(n + 1):
        if i == 1:
            e0.record()
        pipe.deform(bpt, fpt)
    e1.record()
    torch.cuda.synchronize()
    print(f"deform ms per 32-frame batch: {e0.elapsed_time(e1) / max(n, 1):.4f}", flush=True)


if __name__ == "__main__":
    main()
