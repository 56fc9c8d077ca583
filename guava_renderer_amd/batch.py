"""Batched multi-frame rasterization (gsr_forward_batch / gsr_backward_batch).

Replaces the per-frame Python loop of models/UbodyAvatar/gaussian_render.py:37-67: B frames
(views / poses) of one avatar go through one launch per stage with a preallocated workspace and
no host synchronisation, so a whole batch can also be captured in a HIP graph.  Per-frame
attributes may be shared (stride 0: a [P,k] tensor) or per frame (a [B,P,k] tensor).
"""
import ctypes
import weakref

import torch

from . import _lib

C = 32
STAGES = ("preprocess", "scan", "depth_sort", "chunk_count", "tile_scan", "ordered_scatter", "render_fwd",
          "render_bwd", "preprocess_bwd")


def _frame_arg(t, B, P, per, name, device, align16=False):
    """(tensor, element stride between frames) of a shared [P,per] or per-frame [B,P,per] float32
    input on `device`.  The frame stride is the tensor's own stride(0) -- 0 for an expanded tensor,
    whose frames all read one [P,per] table (deform.py's features_color / opacity); rows that are
    not dense in memory are made contiguous first.  align16: every frame's rows start 16-byte
    aligned (the render kernels' feature loads)."""
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a tensor")
    if t.device != device:
        raise ValueError(f"{name} must be on {device} (got {t.device})")
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32 (got {t.dtype})")
    if t.dim() == 2:
        if tuple(t.shape) != (P, per):
            raise ValueError(f"{name}: expected [{P},{per}] or [{B},{P},{per}], got {list(t.shape)}")
        t = t.contiguous()
        return t, 0
    if t.dim() != 3 or tuple(t.shape) != (B, P, per):
        raise ValueError(f"{name}: expected [{P},{per}] or [{B},{P},{per}], got {list(t.shape)}")
    if t.stride(0) == 0:  # one table for every frame (expand)
        row = t[0]
        if not row.is_contiguous():
            row = row.contiguous()
        return row, 0
    dense_rows = t.stride(2) == 1 and (t.stride(1) == per or P == 1)
    fs = t.stride(0)
    if not dense_rows or fs < P * per or (align16 and (fs % 4 or t.data_ptr() % 16)):
        t = t.contiguous()
        fs = P * per
    return t, fs


def _frame_mat(t, B, n, name, device):
    """[B,n] float32 per-frame matrix (viewmatrices / projmatrices [B,16], tanfov [B,2])."""
    if t.device != device or t.dtype != torch.float32:
        raise ValueError(f"{name} must be float32 on {device}")
    if t.numel() != B * n:
        raise ValueError(f"{name}: expected {B}x{n} floats, got shape {list(t.shape)}")
    return t.contiguous()


class BatchRasterizer:
    """Holds the workspace for B frames of P Gaussians at W x H with room for R_capacity
    Gaussian-tile instances.

    Capacity: a forward whose batch needs more than R_capacity instances renders nothing (its
    images are NaN) and sets the workspace's sticky overflow word.  No host synchronisation is
    needed to notice it: after every forward the sticky words are copied asynchronously to pinned
    memory, and the next forward/backward (or poll()) raises CapacityError once that copy has
    landed; poll(wait=True) or status() check at once.

    numerics: the flag word of this rasterizer's calls (include/gsr.h GSR_NUMERICS_*, built by
    _lib.numerics()); 0, the default, is bit-identical to the CPU oracle.  A call may override it
    (forward / backward `numerics=`); nothing is process-wide."""

    def __init__(self, B, P, W, H, R_capacity=None, device="cuda", numerics=0):
        self.B, self.P, self.W, self.H = int(B), int(P), int(W), int(H)
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.R_capacity = int(R_capacity if R_capacity is not None else 16 * P * B)
        self.numerics = int(numerics)
        self.L = _lib.load()
        nbytes = self.L.gsr_batch_workspace_bytes(self.B, self.P, self.W, self.H, self.R_capacity)
        soff = self.L.gsr_batch_status_offset(self.B, self.P, self.W, self.H, self.R_capacity)
        self.workspace = torch.empty((nbytes,), dtype=torch.uint8, device=self.device)
        self._sticky = self.workspace[soff:soff + 16].view(torch.int32)  # include/gsr.h sticky words
        self._sticky.zero_()
        self._overflow = self.workspace[4:8].view(torch.int32).reshape(())  # this call's flag (kCtrlOverflow)
        self._status_host = torch.zeros(4, dtype=torch.int32, pin_memory=True)
        self._status_ev = None
        self.out_color = torch.empty((self.B, C, self.H, self.W), dtype=torch.float32, device=self.device)
        self.out_invdepth = torch.empty((self.B, self.H, self.W), dtype=torch.float32, device=self.device)
        self.radii = torch.empty((self.B, self.P), dtype=torch.int32, device=self.device)

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _inputs(self, means3D, colors, opacities, scales, rotations, viewmatrices, projmatrices,
                tanfov, backgrounds):
        B, P, dev = self.B, self.P, self.device
        none = (None, 0)  # geometry the fused avatar forward assembles on the device
        m, sm = none if means3D is None else _frame_arg(means3D, B, P, 3, "means3D", dev)
        c, sc = _frame_arg(colors, B, P, C, "colors", dev, align16=True)
        o, so = _frame_arg(opacities, B, P, 1, "opacities", dev)
        s, ss = none if scales is None else _frame_arg(scales, B, P, 3, "scales", dev)
        r, sr = none if rotations is None else _frame_arg(rotations, B, P, 4, "rotations", dev)
        v = _frame_mat(viewmatrices, B, 16, "viewmatrices", dev)
        pm = _frame_mat(projmatrices, B, 16, "projmatrices", dev)
        tf = _frame_mat(tanfov, B, 2, "tanfov", dev)
        if backgrounds.device != dev or backgrounds.dtype != torch.float32:
            raise ValueError(f"backgrounds must be float32 on {dev}")
        if backgrounds.dim() == 2:
            if tuple(backgrounds.shape) != (B, C):
                raise ValueError(f"backgrounds: expected [{C}] or [{B},{C}], got {list(backgrounds.shape)}")
            bg = backgrounds.contiguous() if backgrounds.stride(0) != 0 else backgrounds[0].contiguous()
            bs = C if backgrounds.stride(0) != 0 else 0
        elif tuple(backgrounds.shape) == (C,):
            bg, bs = backgrounds.contiguous(), 0
        else:
            raise ValueError(f"backgrounds: expected [{C}] or [{B},{C}], got {list(backgrounds.shape)}")
        keep = (m, c, o, s, r, v, pm, tf, bg)  # alive until the launches are enqueued
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        args = (B, P, self.W, self.H, ptr(m), sm, c.data_ptr(), sc, o.data_ptr(), so, ptr(s), ss, ptr(r), sr)
        return keep, args, (v.data_ptr(), pm.data_ptr(), tf.data_ptr(), bg.data_ptr(), bs)

    def _after_forward(self):
        """Queue the asynchronous copy of the sticky status words (no host synchronisation)."""
        self._status_host.copy_(self._sticky, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._status_ev = ev

    def poll(self, wait=False):
        """Raise CapacityError if a forward enqueued so far overflowed the capacity.  Without
        `wait` this only reads the status copy of the forwards that have already completed."""
        ev = self._status_ev
        if ev is None:
            return
        if wait:
            ev.synchronize()
        elif not ev.query():
            return
        if int(self._status_host[0]):
            rmax = int(self._status_host[1]) & 0xFFFFFFFF
            self.overflow_need = max(getattr(self, "overflow_need", 0), rmax)
            self._sticky.zero_()
            self._status_host.zero_()
            raise _lib.CapacityError(
                f"batch needed {rmax} Gaussian-tile instances, workspace holds {self.R_capacity} "
                f"(that forward's images are NaN); allocate a BatchRasterizer with a larger R_capacity")

    def max_instances_seen(self):
        """Largest batch instance count of the forwards whose status copy has landed (including
        the overflowing ones poll() reported)."""
        return max(int(self._status_host[1]) & 0xFFFFFFFF, getattr(self, "overflow_need", 0))

    def overflow_flag(self):
        """0-dim int32 device tensor: 1 if the last forward overflowed (read on the device, e.g. as an
        optimizer's found_inf), no host synchronisation."""
        return self._overflow

    def forward(self, means3D, colors, opacities, scales, rotations, viewmatrices, projmatrices,
                tanfov, backgrounds, scale_modifier=1.0, antialiasing=False, refine=None, numerics=None,
                forward_only=False):
        """Render B frames.  refine: optional RefineHead -- the refiner's first 1x1 conv + leaky ReLU
        fused into the render epilogue (include/gsr.h gsr_refine_epilogue); its output is
        refine.out [B,n_out,H,W] and only out_color[:, :refine.keep_channels] is written.
        forward_only: no backward() will follow (inference; include/gsr.h GSR_FORWARD_ONLY): the
        workspace skips the rows only the backward reads; the images are the same."""
        self.poll()
        nm = self.numerics if numerics is None else int(numerics)
        if forward_only:
            nm |= _lib.FORWARD_ONLY
        self._fwd_only = bool(forward_only)
        keep, head, (v, pm, tf, bg, bs) = self._inputs(means3D, colors, opacities, scales, rotations,
                                                       viewmatrices, projmatrices, tanfov, backgrounds)
        args = head + (float(scale_modifier), v, pm, tf, bg, bs, self.workspace.data_ptr(), self.R_capacity,
                       self.out_color.data_ptr(), self.out_invdepth.data_ptr(), self.radii.data_ptr(),
                       int(bool(antialiasing)))
        if refine is None:
            _lib.check(self.L.gsr_forward_batch(*args, nm, self._stream()), "gsr_forward_batch")
        else:
            # composite the pre-contracted rows (include/gsr.h gsr_refine_prepare): features and
            # backgrounds both go through the head's 32 -> keep + n_out map
            pc = refine.prepare(keep[1], self._stream())
            bgrows = keep[8].reshape(-1, C)
            pb = refine.prepare(bgrows, self._stream(), cache=False)
            args = list(args)
            args[6] = pc.data_ptr()
            args[18] = pb.data_ptr()
            ep = refine.epilogue(self.B, self.H, self.W)
            _lib.check(self.L.gsr_forward_batch_refine(*args, ctypes.byref(ep), nm, self._stream()),
                       "gsr_forward_batch_refine")
        del keep
        self._after_forward()
        return self.out_color, self.out_invdepth, self.radii

    def forward_deformed(self, deformer, verts, vert_transforms, viewmatrices, projmatrices, tanfov, backgrounds,
                         scale_modifier=1.0, antialiasing=False, numerics=None):
        """The avatar pipeline's fused forward (include/gsr_deform.h gsr_forward_batch_deformed): the
        B frames of `deformer` (deform.GaussianDeformer) on the deformed mesh verts [B,V,3] /
        vert_transforms [B,V,4,4], rendered without materialising the deformed Gaussians (their
        assembly feeds the projection in registers).  Same images as deformer.forward() + forward();
        forward-only (a backward() after it raises)."""
        self.poll()
        nm = self.numerics if numerics is None else int(numerics)
        self._fwd_only = True
        dfm = deformer
        B, P = self.B, self.P
        if dfm.V + dfm.N != P:
            raise ValueError(f"deformer has {dfm.V + dfm.N} Gaussians, the rasterizer {P}")
        if tuple(verts.shape) != (B, dfm.V, 3) or tuple(vert_transforms.shape) != (B, dfm.V, 4, 4):
            raise ValueError("verts / vert_transforms: expected [B,V,3] / [B,V,4,4]")
        # every pointer below goes straight to the kernel: a host (or other-device) tensor must not
        # reach it
        for name, t_ in (("verts", verts), ("vert_transforms", vert_transforms), ("deformer.faces", dfm.faces),
                         ("deformer.colors", dfm.colors), ("deformer.bind", dfm.bind)):
            if t_.device != self.device:
                raise ValueError(f"{name} is on {t_.device}, the rasterizer on {self.device}")
        vb = verts.detach().to(torch.float32).contiguous()
        vt = vert_transforms.detach().to(torch.float32).contiguous()
        keep, head, (v, pm, tf, bg, bs) = self._inputs(None, dfm.colors, dfm.opacity, None, None, viewmatrices,
                                                       projmatrices, tanfov, backgrounds)
        di = _lib.DeformInputs(dfm.V, dfm.faces.shape[0], dfm.N, 0, vb.data_ptr(), vt.data_ptr(),
                               dfm.faces.data_ptr(), dfm.v_rot.data_ptr(), 0, dfm.v_scale.data_ptr(), 0,
                               dfm.bind.data_ptr(), dfm.bary.data_ptr(), dfm.u_local.data_ptr(), 0,
                               dfm.u_rot.data_ptr(), 0, dfm.u_scale.data_ptr(), 0, dfm.bad.data_ptr())
        _lib.check(self.L.gsr_forward_batch_deformed(
            B, self.W, self.H, ctypes.byref(di), head[6], head[7], head[8], head[9], float(scale_modifier),
            v, pm, tf, bg, bs, self.workspace.data_ptr(), self.R_capacity, self.out_color.data_ptr(),
            self.out_invdepth.data_ptr(), self.radii.data_ptr(), int(bool(antialiasing)), nm, self._stream()),
            "gsr_forward_batch_deformed")
        del keep, vb, vt
        self._after_forward()
        return self.out_color, self.out_invdepth, self.radii

    def backward(self, means3D, colors, opacities, scales, rotations, viewmatrices, projmatrices,
                 tanfov, backgrounds, dL_dcolor, dL_dinvdepth=None, scale_modifier=1.0,
                 antialiasing=False, shared=False, numerics=None):
        """Gradients of the last forward, per frame: dict of [B,P,k] tensors (all zero when that
        forward overflowed the capacity; the overflow is reported by the next forward / poll).
        shared=True (attributes shared by every frame, e.g. one avatar under B cameras): the
        attribute gradients summed over the frames instead, dict of [P,k] tensors (means3D, colors,
        opacity, scales, rotations) -- gsr_backward_batch_shared, no [B,P,k] buffers."""
        B, P = self.B, self.P
        if getattr(self, "_fwd_only", False):
            raise _lib.GsrError("backward after forward(forward_only=True): the workspace holds no backward rows")
        nm = self.numerics if numerics is None else int(numerics)
        o = dict(dtype=torch.float32, device=self.device)
        keep, head, (v, pm, tf, bg, bs) = self._inputs(means3D, colors, opacities, scales, rotations,
                                                       viewmatrices, projmatrices, tanfov, backgrounds)
        if tuple(dL_dcolor.shape) != (B, C, self.H, self.W):
            raise ValueError(f"dL_dcolor: expected [{B},{C},{self.H},{self.W}], got {list(dL_dcolor.shape)}")
        dLc = dL_dcolor.to(torch.float32).contiguous()
        dLi = None
        if dL_dinvdepth is not None:
            if dL_dinvdepth.numel() != B * self.H * self.W:
                raise ValueError("dL_dinvdepth: expected [B,H,W]")
            dLi = dL_dinvdepth.to(torch.float32).contiguous()
        if shared:
            # the frame-reduced kernels read ONE attribute row set: per-frame inputs would come back
            # as a single sum over distinct tensors, so they are refused here
            strides = head[5::2]  # means3D, colors, opacities, scales, rotations frame strides
            if any(st_ != 0 for st_ in strides):
                raise ValueError("backward(shared=True) needs attributes shared by every frame "
                                 "([P,k] tensors or frame stride 0); got per-frame inputs")
            g = dict(colors=torch.zeros((P, C), **o), opacity=torch.empty((P, 1), **o),
                     means3D=torch.empty((P, 3), **o), scales=torch.empty((P, 3), **o),
                     rotations=torch.empty((P, 4), **o))
            rc = self.L.gsr_backward_batch_shared(
                *head, float(scale_modifier), v, pm, tf, bg, bs, self.workspace.data_ptr(), self.R_capacity,
                dLc.data_ptr(), dLi.data_ptr() if dLi is not None else None, g["opacity"].data_ptr(),
                g["colors"].data_ptr(), g["means3D"].data_ptr(), g["scales"].data_ptr(),
                g["rotations"].data_ptr(), int(bool(antialiasing)), nm, self._stream())
            _lib.check(rc, "gsr_backward_batch_shared")
            del keep
            return g
        g = dict(mean2D=torch.zeros((B, P, 3), **o), conic=torch.zeros((B, P, 4), **o),
                 opacity=torch.zeros((B, P, 1), **o), colors=torch.zeros((B, P, C), **o),
                 invdepth=torch.zeros((B, P, 1), **o) if dL_dinvdepth is not None else None,
                 means3D=torch.zeros((B, P, 3), **o), cov3D=torch.zeros((B, P, 6), **o),
                 scales=torch.zeros((B, P, 3), **o), rotations=torch.zeros((B, P, 4), **o))
        rc = self.L.gsr_backward_batch(
            *head, float(scale_modifier), v, pm, tf, bg, bs, self.workspace.data_ptr(), self.R_capacity,
            dLc.data_ptr(), dLi.data_ptr() if dLi is not None else None,
            g["mean2D"].data_ptr(), g["conic"].data_ptr(), g["opacity"].data_ptr(),
            g["colors"].data_ptr(), g["invdepth"].data_ptr() if g["invdepth"] is not None else None,
            g["means3D"].data_ptr(), g["cov3D"].data_ptr(), g["scales"].data_ptr(),
            g["rotations"].data_ptr(), int(bool(antialiasing)), nm, self._stream())
        _lib.check(rc, "gsr_backward_batch")
        del keep
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
        self._outs = {}
        self._prep_key, self._prep = None, None

    @classmethod
    def from_conv(cls, conv, negative_slope=0.2, keep_channels=4):
        return cls(conv.weight, conv.bias, negative_slope, keep_channels)

    def prepare(self, rows, stream, cache=True):
        """[..., 32] feature rows -> the pre-contracted rows the refine epilogue composites.  Cached
        for the same tensor OBJECT at the same version (an avatar's features are static across
        frames): a different tensor -- even one the allocator placed at the same address -- or an
        in-place torch update is recomputed.  Writes that bypass torch's version counter (a HIP
        kernel writing through data_ptr()) need invalidate()."""
        # identity: the tensor that owns the memory (a view's base) -- alive while the weakref is,
        # so its address cannot be reused -- plus the view's address, shape and the version counter
        owner = rows._base if rows._base is not None else rows
        ident = (rows.data_ptr(), tuple(rows.shape), rows._version)
        if cache and self._prep_key is not None:
            ref, key = self._prep_key
            if ref() is owner and key == ident:
                return self._prep
        out = torch.empty_like(rows)
        n = rows.numel() // C
        _lib.check(_lib.load().gsr_refine_prepare(n, rows.data_ptr(), self.weight.data_ptr(), self.n_out,
                                                  self.keep_channels, out.data_ptr(), stream),
                   "gsr_refine_prepare")
        if cache:
            self._prep_key, self._prep = (weakref.ref(owner), ident), out
        return out

    def invalidate(self):
        """Drop the cached pre-contracted features (after writing them outside torch's tracking)."""
        self._prep_key, self._prep = None, None

    def epilogue(self, B, H, W):
        """The C-ABI epilogue block; the output tensor is per (stream, shape), so batches in flight
        on different streams do not share one buffer.  self.out is the one of the last call."""
        shape = (B, self.n_out, H, W)
        key = (torch.cuda.current_stream(self.weight.device).cuda_stream, shape)
        out = self._outs.get(key)
        if out is None:
            out = self._outs[key] = torch.empty(shape, dtype=torch.float32, device=self.weight.device)
        self.out = out
        return _lib.RefineEpilogue(self.weight.data_ptr(),
                                   self.bias.data_ptr() if self.bias is not None else None,
                                   self.n_out, self.slope, out.data_ptr(), self.keep_channels)


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
            "gaussians_staged", "list_entries", "tiles_rendered", "dead_ksteps")


def render_counters(fn, device="cuda"):
    """Run `fn()` (one or more forwards) with the instrumented render kernel and return the work
    counters of include/gsr.h:gsr_render_counters as a dict."""
    L = _lib.load()
    buf = torch.zeros(len(COUNTERS), dtype=torch.int64, device=device)
    L.gsr_render_counters(buf.data_ptr())
    try:
        fn()
        torch.cuda.synchronize(device)
    finally:
        L.gsr_render_counters(None)
    v = buf.cpu().tolist()
    return {k: int(v[i]) for i, k in enumerate(COUNTERS)}
