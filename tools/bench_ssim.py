"""fused-SSIM at the reference's own benchmark configuration (submodules/fused-ssim/tests/genplot.py:
B = 5, CH = 1, random images, 50 iterations, wall time per iteration around a synchronize): one
training iteration (forward + backward) and one inference forward (train=False), at 1500 x 1500
(the largest size of the reference's sweep, where its README plot puts an RTX 3080 Ti at about
3 ms and 1.3 ms).  Also per-kernel device times from HIP events.  Prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from fused_ssim import fused_ssim
    torch.manual_seed(0)
    B, CH, iters = 5, 1, 50
    out = {"workload": "fused-ssim genplot.py config", "B": B, "CH": CH, "iterations": iters, "sizes": {}}
    for d in (512, 1000, 1500):
        img1 = torch.nn.Parameter(torch.rand([B, CH, d, d], device="cuda"))
        img2 = torch.rand([B, CH, d, d], device="cuda")
        for _ in range(5):  # warm-up
            fused_ssim(img1, img2).backward()
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(iters):
            v = fused_ssim(img1, img2)
            v.backward()
        torch.cuda.synchronize()
        train_ms = (time.time() - t0) / iters * 1000
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fused_ssim(img1, img2).backward()
        e1.record()
        torch.cuda.synchronize()
        train_dev_ms = e0.elapsed_time(e1) / iters
        with torch.no_grad():
            for _ in range(5):
                fused_ssim(img1, img2, train=False)
            torch.cuda.synchronize()
            t0 = time.time()
            for _ in range(iters):
                fused_ssim(img1, img2, train=False)
            torch.cuda.synchronize()
            infer_ms = (time.time() - t0) / iters * 1000
        # bytes: fwd reads 2 images + writes the map and 3 partials (train); bwd reads 2 images +
        # 3 partials + dL/dmap, writes dL/dimg1
        px = B * CH * d * d
        out["sizes"][str(d)] = {"train_iter_ms": round(train_ms, 4), "train_iter_device_ms": round(train_dev_ms, 4),
                                "inference_ms": round(infer_ms, 4),
                                "train_GBs_min_traffic": round(px * 4 * (6 + 7) / (train_dev_ms * 1e-3) / 1e9, 1)}
    out["reference_published"] = {"gpu": "RTX 3080 Ti (README plot, genplot.py)", "train_iter_ms_1500": 3.0,
                                  "inference_ms_1500": 1.3}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
