"""Rasterizer training step (BASELINE config 4): forward + backward raster + fused-SSIM loss.

One step over the B frames of this rank (main/trainer.py:82-102 does, per iteration: render the
batch, Optimization_Loss, fabric.backward -> DDP gradient all-reduce, Adam step):
  1. BatchRasterizer.forward of the shared Gaussian attributes for B cameras (one launch set);
  2. loss = (1 - lambda) * L1 + lambda * (1 - fused_ssim) of the raw RGB channels + L1 of a refined image
     made from ALL 32 channels (the reference's `renders` term, :92; its StyleUNet refiner is out
     of scope, so a fixed random 1x1 conv 32 -> 3 stands in), so every feature channel carries a
     gradient into the rasterizer backward as in the reference's training; the L1 terms and the
     gradient assembly are one gfx950 pass (gsr_image_loss).  The reference's raw_renders term
     (utils/loss_utils.py:116-119) is lambda_l1 * L1 + an LPIPS perceptual term; LPIPS (AlexNet with
     weights fetched from a URL) is out of scope, and fused-SSIM -- the reference's own native loss
     kernel, BASELINE config 4 -- stands in for that perceptual term;
  3. BatchRasterizer.backward(shared=True) (render_bwd + cov/preprocess backward kernels) -> the
     shared attributes' gradients [P,k], summed over the frames inside the kernels (no [B,P,k]
     buffers);
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
import ctypes
import os
import warnings

import torch
import torch.distributed as dist

from . import _lib, parallel
from .batch import BatchRasterizer
from .fused_ssim import fused_ssim

C = 32


class SplatTrainer:
    def __init__(self, params, B, W, H, R_capacity, device="cuda", lr=1e-3, lambda_ssim=0.2, refine_head=True,
                 numerics=0):
        """params: dict of float32 device tensors means3D [P,3], colors [P,32], opacities [P,1],
        scales [P,3], rotations [P,4] (made leaves with requires_grad).  refine_head=False: the loss
        sees the RGB channels only.  numerics: the rasterizer calls' GSR_NUMERICS_* flags."""
        self.dev = torch.device(device)
        self.p = {k: v.detach().clone().contiguous().requires_grad_(True) for k, v in params.items()}
        P = self.p["means3D"].shape[0]
        self.numerics = int(numerics)
        self.rast = BatchRasterizer(B, P, W, H, R_capacity=R_capacity, device=self.dev, numerics=self.numerics)
        self.opt = torch.optim.Adam(list(self.p.values()), lr=lr, fused=True)
        self.skipped_steps = 0
        self.B, self.W, self.H = B, W, H
        self.lambda_ssim = lambda_ssim
        self.bg = torch.zeros((B, C), dtype=torch.float32, device=self.dev)
        self.dinv = torch.zeros((B, H, W), dtype=torch.float32, device=self.dev)  # materialised, as autograd does
        g = torch.Generator().manual_seed(11)
        self.refine_w = ((torch.rand((3, C), generator=g) * 2 - 1) / C ** 0.5).to(self.dev) if refine_head else None
        self.shared_backward = os.environ.get("GSR_TRAIN_PERFRAME") != "1"  # "1": per-frame grads + sum (A/B)
        self._loss_bufs = None  # (per-workgroup loss partials, dL/dfeatures [B,32,H,W])

    def _grow(self, err):
        """An earlier step overflowed (and was skipped on the device): grow the workspace to 1.5x the
        instance count that step needed (at least double)."""
        self.skipped_steps += 1
        old = self.rast
        cap = max(int(old.max_instances_seen() * 1.5), 2 * old.R_capacity) + 1024
        warnings.warn(f"SplatTrainer: {err}; step skipped, R capacity {old.R_capacity} -> {cap}")
        self.rast = BatchRasterizer(old.B, old.P, old.W, old.H, R_capacity=cap, device=self.dev,
                                    numerics=self.numerics)
        del old

    def gradients(self, views, projs, tanf, target):
        """Forward + loss + backward of one step: (loss, dict of the attributes' gradients summed
        over this rank's frames), before any all-reduce or update."""
        want = (self.B, 3, self.H, self.W)
        if tuple(target.shape) != want or target.device != self.dev:
            raise ValueError(f"target: expected {list(want)} on {self.dev}, got {list(target.shape)} on {target.device}")
        try:
            self.rast.poll()
        except _lib.CapacityError as e:
            self._grow(e)
        p = self.p
        col, _, _ = self.rast.forward(p["means3D"].detach(), p["colors"].detach(), p["opacities"].detach(),
                                      p["scales"].detach(), p["rotations"].detach(), views, projs, tanf,
                                      self.bg)
        # SSIM term through autograd (fused_ssim kernels); the two L1 terms, their gradient and the
        # SSIM gradient's addition in one pass over the 32-channel frames (gsr_image_loss)
        img = col[:, :3].detach().requires_grad_(True)
        ssim_term = self.lambda_ssim * (1.0 - fused_ssim(img, target))
        ssim_term.backward()
        tgt = target.detach().to(torch.float32).contiguous()
        B, _, H, W = col.shape
        L = _lib.load()
        n_part = L.gsr_image_loss_partials(B, H, W)
        if self._loss_bufs is None or self._loss_bufs[0].shape[0] != n_part:
            self._loss_bufs = (torch.empty((n_part,), dtype=torch.float32, device=self.dev),
                               torch.empty_like(col))
        part, dL = self._loss_bufs
        _lib.check(L.gsr_image_loss(B, H, W, col.data_ptr(), tgt.data_ptr(),
                                    self.refine_w.data_ptr() if self.refine_w is not None else None,
                                    1.0 - self.lambda_ssim, 1.0 if self.refine_w is not None else 0.0,
                                    img.grad.contiguous().data_ptr(), dL.data_ptr(), part.data_ptr(),
                                    ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)),
                   "gsr_image_loss")
        loss = ssim_term.detach() + part.sum()
        g = self.rast.backward(p["means3D"].detach(), p["colors"].detach(), p["opacities"].detach(),
                               p["scales"].detach(), p["rotations"].detach(), views, projs, tanf, self.bg,
                               dL, self.dinv, shared=self.shared_backward)
        if not self.shared_backward:
            g = {k: v.sum(0) for k, v in g.items() if v is not None and v.dim() == 3}
        grads = {"means3D": g["means3D"], "colors": g["colors"], "opacities": g["opacity"],
                 "scales": g["scales"], "rotations": g["rotations"]}
        return loss.detach(), grads

    def rgb_loss(self, img, target):
        """(1 - lambda) L1 + lambda (1 - SSIM) of the raw RGB channels [B,3,H,W]."""
        return (1.0 - self.lambda_ssim) * (img - target).abs().mean() + \
            self.lambda_ssim * (1.0 - fused_ssim(img, target))

    def loss(self, feat, target):
        """The step's loss of rendered features [B,32,H,W] against RGB targets [B,3,H,W]."""
        loss = self.rgb_loss(feat[:, :3], target)
        if self.refine_w is not None:
            loss = loss + (torch.einsum("oc,bchw->bohw", self.refine_w, feat) - target).abs().mean()
        return loss

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
