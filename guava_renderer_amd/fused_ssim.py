"""Fused SSIM on gfx950 with the reference's Python API (submodules/fused-ssim/fused_ssim/__init__.py).

  fusedssim(C1, C2, img1, img2, train)  -> (ssim_map, dm_dmu1, dm_dsigma1_sq, dm_dsigma12)
                                           (the reference's fused_ssim_cuda.fusedssim, ssim.cu:368-404)
  fusedssim_backward(C1, C2, img1, img2, dL_dmap, dm_dmu1, dm_dsigma1_sq, dm_dsigma12) -> dL_dimg1
                                           (ssim.cu:406-444)
  FusedSSIMMap                            autograd.Function (__init__.py:8-34)
  fused_ssim(img1, img2, padding="same", train=True) -> mean SSIM (__init__.py:36-41)

Kernels: csrc/ssim.hip through include/gsr_ssim.h.  GPU only: CPU tensors raise.
"""
import ctypes

import torch

from . import _lib

allowed_padding = ["same", "valid"]


def _check(img):
    if not img.is_cuda:
        raise RuntimeError("fused_ssim runs on the GPU only (got a CPU tensor)")
    if img.dim() != 4:
        raise RuntimeError(f"fused_ssim expects [B, CH, H, W] images, got {tuple(img.shape)}")


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def fusedssim(C1, C2, img1, img2, train):
    _check(img1)
    _check(img2)
    a = img1.detach().to(torch.float32).contiguous()
    b = img2.detach().to(torch.float32).contiguous()
    B, CH, H, W = a.shape
    ssim_map = torch.empty_like(a)
    if train:
        dmu, ds1, ds12 = torch.empty_like(a), torch.empty_like(a), torch.empty_like(a)
    else:
        e = torch.empty(0, device=a.device)
        dmu = ds1 = ds12 = e
    rc = _lib.load().gsr_fused_ssim(B, CH, H, W, float(C1), float(C2), _p(a), _p(b), _p(ssim_map),
                                    _p(dmu) if train else None, _p(ds1) if train else None,
                                    _p(ds12) if train else None, _stream(a))
    _lib.check(rc, "gsr_fused_ssim")
    return ssim_map, dmu, ds1, ds12


def fusedssim_backward(C1, C2, img1, img2, dL_dmap, dm_dmu1, dm_dsigma1_sq, dm_dsigma12):
    a = img1.detach().to(torch.float32).contiguous()
    b = img2.detach().to(torch.float32).contiguous()
    g = dL_dmap.to(torch.float32).contiguous()
    B, CH, H, W = a.shape
    out = torch.empty_like(a)
    rc = _lib.load().gsr_fused_ssim_backward(B, CH, H, W, float(C1), float(C2), _p(a), _p(b), _p(g),
                                             _p(dm_dmu1.contiguous()), _p(dm_dsigma1_sq.contiguous()),
                                             _p(dm_dsigma12.contiguous()), _p(out), _stream(a))
    _lib.check(rc, "gsr_fused_ssim_backward")
    return out


class FusedSSIMMap(torch.autograd.Function):
    @staticmethod
    def forward(ctx, C1, C2, img1, img2, padding="same", train=True):
        ssim_map, dm_dmu1, dm_dsigma1_sq, dm_dsigma12 = fusedssim(C1, C2, img1, img2, train)
        if padding == "valid":
            ssim_map = ssim_map[:, :, 5:-5, 5:-5]
        ctx.save_for_backward(img1.detach(), img2, dm_dmu1, dm_dsigma1_sq, dm_dsigma12)
        ctx.C1 = C1
        ctx.C2 = C2
        ctx.padding = padding
        return ssim_map

    @staticmethod
    def backward(ctx, opt_grad):
        img1, img2, dm_dmu1, dm_dsigma1_sq, dm_dsigma12 = ctx.saved_tensors
        C1, C2, padding = ctx.C1, ctx.C2, ctx.padding
        dL_dmap = opt_grad
        if padding == "valid":
            dL_dmap = torch.zeros_like(img1)
            dL_dmap[:, :, 5:-5, 5:-5] = opt_grad
        grad = fusedssim_backward(C1, C2, img1, img2, dL_dmap, dm_dmu1, dm_dsigma1_sq, dm_dsigma12)
        return None, None, grad, None, None, None


def fused_ssim(img1, img2, padding="same", train=True):
    C1 = 0.01 ** 2
    C2 = 0.03 ** 2
    assert padding in allowed_padding
    map = FusedSSIMMap.apply(C1, C2, img1, img2, padding, train)  # noqa: A001
    return map.mean()
