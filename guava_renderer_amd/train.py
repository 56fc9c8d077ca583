"""Rasterizer training step (BASELINE config 4): forward + backward raster + fused-SSIM loss.

One step over the B frames of this rank (main/trainer.py:82-102 does, per iteration: render the
batch, Optimization_Loss, fabric.backward -> DDP gradient all-reduce, Adam step):
  1. BatchRasterizer.forward of the shared Gaussian attributes for B cameras (one launch set);
  2. loss = (1 - lambda) * L1 + lambda * (1 - fused_ssim) on the RGB channels against the targets
     (the fused_ssim HIP kernels, guava_renderer_amd/fused_ssim.py);
  3. BatchRasterizer.backward (render_bwd + cov/preprocess backward kernels) -> per-frame
     gradients [B,P,k], summed over frames into the shared attributes' gradients;
  4. world > 1: ONE flat RCCL all-reduce of those gradients (parallel.reduce_shared_grads; the
     reference's DDP all-reduce, trainer.py:40-43,95), averaged over ranks;
  5. Adam on the attributes (fused Adam).
Capacity overflow (more Gaussian-tile instances than the workspace holds, e.g. after the attributes
drifted under the optimizer) needs no host synchronisation to stay harmless: the overflowing
forward renders NaN frames (so the step's loss is NaN), the backward produces no gradient, and the
workspace's overflow flag is the optimizer's `found_inf`, so Adam skips that step on the device
(as GradScaler does for an inf).  The next step sees the flag through the asynchronous status copy,
grows the workspace and counts the step in `skipped_steps`.
The reference trains networks that predict the Gaussians; those networks are out of scope here
(SURVEY.md 2.1), so the trainable parameters are the Gaussian attributes themselves -- the
rasterizer-side work of the step (fwd, bwd, SSIM, all-reduce, update) is the same.
"""
import warnings

import torch
import torch.distributed as dist

from . import _lib, parallel
from .batch import BatchRasterizer
from .fused_ssim import fused_ssim

C = 32


class SplatTrainer:
    def __init__(self, params, B, W, H, R_capacity, device="cuda", lr=1e-3, lambda_ssim=0.2):
        """params: dict of float32 device tensors means3D [P,3], colors [P,32], opacities [P,1],
        scales [P,3], rotations [P,4] (made leaves with requires_grad)."""
        self.dev = torch.device(device)
        self.p = {k: v.detach().clone().contiguous().requires_grad_(True) for k, v in params.items()}
        P = self.p["means3D"].shape[0]
        self.rast = BatchRasterizer(B, P, W, H, R_capacity=R_capacity, device=self.dev)
        self.opt = torch.optim.Adam(list(self.p.values()), lr=lr, fused=True)
        self.skipped_steps = 0
        self.B, self.W, self.H = B, W, H
        self.lambda_ssim = lambda_ssim
        self.bg = torch.zeros((B, C), dtype=torch.float32, device=self.dev)
        self.dL = torch.zeros((B, C, H, W), dtype=torch.float32, device=self.dev)
        self.dinv = torch.zeros((B, H, W), dtype=torch.float32, device=self.dev)  # materialised, as autograd does

    def _grow(self, err):
        """An earlier step overflowed (and was skipped on the device): grow the workspace to 1.5x the
        instance count that step needed (at least double)."""
        self.skipped_steps += 1
        old = self.rast
        cap = max(int(old.max_instances_seen() * 1.5), 2 * old.R_capacity) + 1024
        warnings.warn(f"SplatTrainer: {err}; step skipped, R capacity {old.R_capacity} -> {cap}")
        self.rast = BatchRasterizer(old.B, old.P, old.W, old.H, R_capacity=cap, device=self.dev)
        del old

    def gradients(self, views, projs, tanf, target):
        """Forward + loss + backward of one step: (loss, dict of the attributes' gradients summed
        over this rank's frames), before any all-reduce or update."""
        try:
            self.rast.poll()
        except _lib.CapacityError as e:
            self._grow(e)
        p = self.p
        col, _, _ = self.rast.forward(p["means3D"].detach(), p["colors"].detach(), p["opacities"].detach(),
                                      p["scales"].detach(), p["rotations"].detach(), views, projs, tanf,
                                      self.bg)
        img = col[:, :3].detach().requires_grad_(True)
        loss = (1.0 - self.lambda_ssim) * (img - target).abs().mean() + \
            self.lambda_ssim * (1.0 - fused_ssim(img, target))
        loss.backward()
        self.dL[:, :3].copy_(img.grad)
        g = self.rast.backward(p["means3D"].detach(), p["colors"].detach(), p["opacities"].detach(),
                               p["scales"].detach(), p["rotations"].detach(), views, projs, tanf, self.bg,
                               self.dL, self.dinv)
        grads = {"means3D": g["means3D"].sum(0), "colors": g["colors"].sum(0),
                 "opacities": g["opacity"].sum(0), "scales": g["scales"].sum(0),
                 "rotations": g["rotations"].sum(0)}
        return loss.detach(), grads

    def step(self, views, projs, tanf, target):
        loss, grads = self.gradients(views, projs, tanf, target)
        p = self.p
        # this step's capacity overflow, as the optimizer's found_inf (read on the device)
        ovf = self.rast.overflow_flag().to(torch.float32).reshape(1)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            grads["~overflow"] = ovf  # any rank's overflow skips the step on every rank
            parallel.reduce_shared_grads(grads)
            ovf = grads.pop("~overflow")
            for v in grads.values():
                v.div_(dist.get_world_size())
        for k, v in grads.items():
            p[k].grad = v.reshape(p[k].shape)
        self.opt.found_inf = (ovf > 0).to(torch.float32).reshape(())
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        return loss
