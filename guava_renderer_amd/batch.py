"""Batched multi-frame rasterization (gsr_forward_batch / gsr_backward_batch).

Replaces the per-frame Python loop of models/UbodyAvatar/gaussian_render.py:37-67: B frames
(views / poses) of one avatar go through one launch per stage with a preallocated workspace and
no host synchronisation, so a whole batch can also be captured in a HIP graph.  Per-frame
attributes may be shared (stride 0: a [P,k] tensor) or per frame (a [B,P,k] tensor).
"""
import ctypes

import torch

from . import _lib

C = 32
STAGES = ("preprocess", "scan", "depth_sort", "chunk_count", "tile_scan", "ordered_scatter", "render_fwd",
          "render_bwd", "preprocess_bwd")


def _stride(t, B, per):
    """Element stride between frames for a [P,per] (shared) or [B,P,per] tensor."""
    if t.dim() == 3:
        assert t.shape[0] == B and t.shape[2] == per, t.shape
        return t.shape[1] * per
    assert t.dim() == 2 and t.shape[1] == per, t.shape
    return 0


class BatchRasterizer:
    """Holds the workspace for B frames of P Gaussians at W x H with room for R_capacity
    Gaussian-tile instances."""

    def __init__(self, B, P, W, H, R_capacity=None, device="cuda"):
        self.B, self.P, self.W, self.H = int(B), int(P), int(W), int(H)
        self.device = torch.device(device)
        self.R_capacity = int(R_capacity if R_capacity is not None else 16 * P * B)
        self.L = _lib.load()
        nbytes = self.L.gsr_batch_workspace_bytes(self.B, self.P, self.W, self.H, self.R_capacity)
        self.workspace = torch.empty((nbytes,), dtype=torch.uint8, device=self.device)
        self.out_color = torch.empty((self.B, C, self.H, self.W), dtype=torch.float32, device=self.device)
        self.out_invdepth = torch.empty((self.B, self.H, self.W), dtype=torch.float32, device=self.device)
        self.radii = torch.empty((self.B, self.P), dtype=torch.int32, device=self.device)

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def forward(self, means3D, colors, opacities, scales, rotations, viewmatrices, projmatrices,
                tanfov, backgrounds, scale_modifier=1.0, antialiasing=False, refine=None):
        """Render B frames.  refine: optional RefineHead -- the refiner's first 1x1 conv + leaky ReLU
        fused into the render epilogue (include/gsr.h gsr_refine_epilogue); its output is
        refine.out [B,n_out,H,W] and only out_color[:, :refine.keep_channels] is written."""
        B = self.B
        bg_stride = backgrounds.shape[-1] if backgrounds.dim() == 2 else 0
        args = (B, self.P, self.W, self.H,
                means3D.data_ptr(), _stride(means3D, B, 3), colors.data_ptr(), _stride(colors, B, C),
                opacities.data_ptr(), _stride(opacities, B, 1), scales.data_ptr(), _stride(scales, B, 3),
                rotations.data_ptr(), _stride(rotations, B, 4), float(scale_modifier),
                viewmatrices.data_ptr(), projmatrices.data_ptr(), tanfov.data_ptr(),
                backgrounds.data_ptr(), bg_stride, self.workspace.data_ptr(), self.R_capacity,
                self.out_color.data_ptr(), self.out_invdepth.data_ptr(), self.radii.data_ptr(),
                int(bool(antialiasing)))
        if refine is None:
            _lib.check(self.L.gsr_forward_batch(*args, self._stream()), "gsr_forward_batch")
        else:
            # composite the pre-contracted rows (include/gsr.h gsr_refine_prepare): features and
            # backgrounds both go through the head's 32 -> keep + n_out map
            pc = refine.prepare(colors, self._stream())
            pb = refine.prepare(backgrounds.reshape(-1, C), self._stream(), cache=False)
            args = list(args)
            args[6] = pc.data_ptr()
            args[18] = pb.data_ptr()
            ep = refine.epilogue(B, self.H, self.W)
            _lib.check(self.L.gsr_forward_batch_refine(*args, ctypes.byref(ep), self._stream()),
                       "gsr_forward_batch_refine")
        return self.out_color, self.out_invdepth, self.radii

    def backward(self, means3D, colors, opacities, scales, rotations, viewmatrices, projmatrices,
                 tanfov, backgrounds, dL_dcolor, dL_dinvdepth=None, scale_modifier=1.0,
                 antialiasing=False):
        """Gradients of the last forward, per frame: dict of [B,P,k] tensors."""
        B, P = self.B, self.P
        o = dict(dtype=torch.float32, device=self.device)
        g = dict(mean2D=torch.zeros((B, P, 3), **o), conic=torch.zeros((B, P, 4), **o),
                 opacity=torch.zeros((B, P, 1), **o), colors=torch.zeros((B, P, C), **o),
                 invdepth=torch.zeros((B, P, 1), **o) if dL_dinvdepth is not None else None,
                 means3D=torch.zeros((B, P, 3), **o), cov3D=torch.zeros((B, P, 6), **o),
                 scales=torch.zeros((B, P, 3), **o), rotations=torch.zeros((B, P, 4), **o))
        bg_stride = backgrounds.shape[-1] if backgrounds.dim() == 2 else 0
        rc = self.L.gsr_backward_batch(
            B, P, self.W, self.H,
            means3D.data_ptr(), _stride(means3D, B, 3), colors.data_ptr(), _stride(colors, B, C),
            opacities.data_ptr(), _stride(opacities, B, 1), scales.data_ptr(), _stride(scales, B, 3),
            rotations.data_ptr(), _stride(rotations, B, 4), float(scale_modifier),
            viewmatrices.data_ptr(), projmatrices.data_ptr(), tanfov.data_ptr(),
            backgrounds.data_ptr(), bg_stride, self.workspace.data_ptr(), self.R_capacity,
            dL_dcolor.contiguous().data_ptr(),
            dL_dinvdepth.contiguous().data_ptr() if dL_dinvdepth is not None else None,
            g["mean2D"].data_ptr(), g["conic"].data_ptr(), g["opacity"].data_ptr(),
            g["colors"].data_ptr(), g["invdepth"].data_ptr() if g["invdepth"] is not None else None,
            g["means3D"].data_ptr(), g["cov3D"].data_ptr(), g["scales"].data_ptr(),
            g["rotations"].data_ptr(), int(bool(antialiasing)), self._stream())
        _lib.check(rc, "gsr_backward_batch")
        return g

    def status(self):
        """(R_total, overflow) of the last forward; synchronises the stream."""
        R = ctypes.c_int64(0)
        ovf = ctypes.c_int(0)
        _lib.check(self.L.gsr_batch_status(self.workspace.data_ptr(), self.B, self.P,
                                           ctypes.byref(R), ctypes.byref(ovf), self._stream()),
                   "gsr_batch_status")
        return int(R.value), bool(ovf.value)


class RefineHead:
    """StyleUNet.conv_body_first (nn.Conv2d(32, n_out, 1), styleunet.py:110) + F.leaky_relu_(., 0.2)
    (:178), evaluated inside the render kernel.  weight [n_out,32] or [n_out,32,1,1], bias [n_out]."""

    def __init__(self, weight, bias=None, negative_slope=0.2, keep_channels=4):
        w = weight.detach().reshape(weight.shape[0], -1).to(torch.float32).contiguous()
        assert w.shape[1] == C and 1 <= w.shape[0] <= C, w.shape
        self.weight = w
        self.bias = bias.detach().to(torch.float32).contiguous() if bias is not None else None
        self.n_out = w.shape[0]
        self.slope = float(negative_slope)
        self.keep_channels = int(keep_channels)
        assert self.keep_channels + self.n_out <= C
        self.out = None
        self._prep_key, self._prep = None, None

    @classmethod
    def from_conv(cls, conv, negative_slope=0.2, keep_channels=4):
        return cls(conv.weight, conv.bias, negative_slope, keep_channels)

    def prepare(self, rows, stream, cache=True):
        """[..., 32] feature rows -> the pre-contracted rows the refine epilogue composites; cached
        on the tensor's identity and version (an avatar's features are static across frames)."""
        key = (rows.data_ptr(), tuple(rows.shape), rows._version)
        if cache and self._prep_key == key:
            return self._prep
        out = torch.empty_like(rows)
        n = rows.numel() // C
        _lib.check(_lib.load().gsr_refine_prepare(n, rows.data_ptr(), self.weight.data_ptr(), self.n_out,
                                                  self.keep_channels, out.data_ptr(), stream),
                   "gsr_refine_prepare")
        if cache:
            self._prep_key, self._prep = key, out
        return out

    def epilogue(self, B, H, W):
        shape = (B, self.n_out, H, W)
        if self.out is None or tuple(self.out.shape) != shape:
            self.out = torch.empty(shape, dtype=torch.float32, device=self.weight.device)
        return _lib.RefineEpilogue(self.weight.data_ptr(),
                                   self.bias.data_ptr() if self.bias is not None else None,
                                   self.n_out, self.slope, self.out.data_ptr(), self.keep_channels)


def profile_enable(stages=("render_fwd",)):
    mask = 0
    for s in stages:
        mask |= 1 << STAGES.index(s)
    _lib.load().gsr_profile_enable(mask)


def profile_read():
    n = len(STAGES)
    ms = (ctypes.c_double * n)()
    cnt = (ctypes.c_int * n)()
    _lib.check(_lib.load().gsr_profile_read(ms, cnt, n), "gsr_profile_read")
    return {s: (ms[i], cnt[i]) for i, s in enumerate(STAGES) if cnt[i]}


COUNTERS = ("pairs_evaluated", "pairs_contributing", "strip_pairs_blended", "mfma_ksteps",
            "gaussians_staged", "list_entries", "tiles_rendered")


def render_counters(fn, device="cuda"):
    """Run `fn()` (one or more forwards) with the instrumented render kernel and return the work
    counters of include/gsr.h:gsr_render_counters as a dict."""
    L = _lib.load()
    buf = torch.zeros(8, dtype=torch.int64, device=device)
    L.gsr_render_counters(buf.data_ptr())
    try:
        fn()
        torch.cuda.synchronize(device)
    finally:
        L.gsr_render_counters(None)
    v = buf.cpu().tolist()
    return {k: int(v[i]) for i, k in enumerate(COUNTERS)}
