"""The native `_C` surface of diff_gaussian_rasterization_32, over the gfx950 C ABI (libgsr.so).

Same functions, positional signatures, return tuples and error behaviour as the reference's
pybind module (/root/reference/submodules/diff-gaussian-rasterization-32/ext.cpp:15-19,
rasterize_points.cu:36-124 (forward), :127-223 (backward), :225-244 (mark_visible)).
Tensors are allocated by the torch (HIP) caching allocator; the three scratch buffers are uint8
tensors resized through the C ABI's allocator callbacks, exactly as resizeFunctional does
(rasterize_points.cu:27-33), and handed back to backward by autograd.
Differences by design: scratch buffers live on means3D's device (the reference uses the current
device); kernels run on the current HIP stream of that device.
"""
import collections
import ctypes
import os
import weakref

import torch

from .. import _lib

NUM_CHANNELS = 32
# binning buffers up to this size take the no-sync forward (gsr_forward_async); larger ones (big
# images x many Gaussians) size the buffer from the synchronous R read-back as the reference does.
# The no-sync forward's buffer is the P x tiles bound, so it is only used when nobody keeps the
# buffer (exact_binning=False: inference -- GaussianRasterizer_32 under no_grad drops it with the
# call); a forward whose buffers autograd saves for backward sizes it to the exact R.  A frame's
# buffer holds 8 B per bound instance (list entry + quad mask): 1 GB covers 100k Gaussians at 512^2
# (the bound is P x tiles; the inference path keeps one such arena per stream, of 288 GB of HBM).
ASYNC_BINNING_MB = int(os.environ.get("GSR_ASYNC_BINNING_MB", "1024"))
# numerics of the reference-signature calls that pass none (GaussianRasterizer_32 as GUAVA calls it):
# 0 = bit-identical to the oracle.  A deployment can opt into a tolerance mode for the unchanged
# caller, e.g. GSR_NUMERICS=split_bf16 (or fast_exp), comma-separated.
_NUMERICS_NAMES = {"fast_exp": 1, "split_bf16": 2}
DEFAULT_NUMERICS = 0
for _n in filter(None, (x.strip() for x in os.environ.get("GSR_NUMERICS", "").split(","))):
    if _n not in _NUMERICS_NAMES:
        raise ValueError(f"GSR_NUMERICS: unknown flag {_n!r} (known: {sorted(_NUMERICS_NAMES)})")
    DEFAULT_NUMERICS |= _NUMERICS_NAMES[_n]


class PendingCount:
    """num_rendered of a forward that did not wait for the device (gsr_forward_async): reading it
    (int(), comparisons, arithmetic, printing) waits for that forward and raises the reference's
    errors (a culled point with prefiltered set, an instance count beyond 2^31 - 1) then."""
    __slots__ = ("_status", "_event", "_value", "_error", "__weakref__")

    def __init__(self, status, event):
        self._status, self._event, self._value, self._error = status, event, None, None

    def _resolve(self):
        """Wait for the forward and take its status out of the (reused) pinned slot; an error is
        kept for THIS count's readers, never raised into whoever triggered the resolution."""
        if self._value is None and self._error is None:
            self._event.synchronize()
            r, ovf, err = (int(x) for x in self._status[:3].tolist())
            if err & 1:
                self._error = RuntimeError("Point is filtered although prefiltered is set. This shouldn't happen!")
            elif ovf:
                self._error = _lib.CapacityError("instance count exceeds 2^31 - 1 (num_rendered is an int)")
            else:
                self._value = r

    def __int__(self):
        self._resolve()
        if self._error is not None:
            raise self._error
        return self._value

    __index__ = __int__

    def __eq__(self, o):
        return int(self) == o

    def __lt__(self, o):
        return int(self) < o

    def __le__(self, o):
        return int(self) <= o

    def __gt__(self, o):
        return int(self) > o

    def __ge__(self, o):
        return int(self) >= o

    def __hash__(self):
        return hash(int(self))

    def __bool__(self):
        return int(self) != 0

    def __add__(self, o):
        return int(self) + o

    __radd__ = __add__

    def __mul__(self, o):
        return int(self) * o

    __rmul__ = __mul__

    def __sub__(self, o):
        return int(self) - o

    def __rsub__(self, o):
        return o - int(self)

    def __floordiv__(self, o):
        return int(self) // o

    def __mod__(self, o):
        return int(self) % o

    def __neg__(self):
        return -int(self)

    def __repr__(self):
        return repr(int(self))

    __str__ = __repr__

    def __format__(self, spec):
        return format(int(self), spec)


class _StatusRing:
    """Pinned 16-byte status slots for gsr_forward_async, reused round-robin.  A slot is handed out
    again only after its copy has landed and its PendingCount (if still alive) has read it, so a
    pending device-to-host copy never writes memory that belongs to someone else."""

    def __init__(self, n=256):
        self.buf = torch.zeros((n, 4), dtype=torch.int32, pin_memory=True)
        self.owner = [None] * n  # (event, weakref to PendingCount)
        self.i = 0

    def take(self, stream):
        k = self.i
        self.i = (k + 1) % self.buf.shape[0]
        prev = self.owner[k]
        if prev is not None:
            ev, ref = prev
            pc = ref()
            if pc is not None:
                pc._resolve()  # take its status out of this slot before the slot is rewritten
            else:
                ev.synchronize()
        ev = torch.cuda.Event()
        slot = self.buf[k]
        return slot, ev, k

    def bind(self, k, ev, pc):
        self.owner[k] = (ev, weakref.ref(pc))


_RINGS = {}


def _ptr(t):
    """Device pointer of a tensor, or None for an empty tensor (reference: data<float>() of an
    empty tensor is nullptr)."""
    if t is None or t.numel() == 0:
        return None
    return t.data_ptr()


def _dev_f32(t, device, name):
    if t is None or t.numel() == 0:
        return t
    if t.device != device:
        raise RuntimeError(f"{name} must be on {device} (got {t.device})")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32 (got {t.dtype})")
    return t.contiguous()


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class _Resizer:
    """Holds a growable uint8 tensor; called by the C ABI with the requested size."""

    def __init__(self, device):
        self.t = torch.empty((0,), dtype=torch.uint8, device=device)
        self.cb = _lib.ALLOC_FN(self._cb)

    def _cb(self, ctx, n):
        self.t.resize_((int(n),))
        return self.t.data_ptr()


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier,
                        cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height,
                        image_width, sh, degree, campos, prefiltered, antialiasing, debug, *, numerics=None,
                        exact_binning=False):
    """RasterizeGaussiansCUDA (rasterize_points.cu:36-124).  Returns
    (num_rendered, color[32,H,W], radii[P] int32, geomBuffer, binningBuffer, imgBuffer, invdepth[1,H,W]).
    numerics (keyword only, not in the reference): the call's GSR_NUMERICS_* flags (_lib.numerics());
    the default 0 is bit-identical to the CPU oracle.
    exact_binning (keyword only): size binningBuffer to the exact instance count after a host read-back
    of num_rendered (the reference's behaviour, rasterizer_impl.cu:279-291) -- for buffers kept until
    backward.  Otherwise (default) the forward does not wait for the device: binningBuffer is the
    P x tiles bound (4 B per possible instance; R cannot exceed it) and num_rendered a PendingCount."""
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    if numerics is None:
        numerics = DEFAULT_NUMERICS
    P = int(means3D.size(0))
    H = int(image_height)
    W = int(image_width)
    dev = means3D.device
    fopts = dict(dtype=torch.float32, device=dev)
    # the render pass writes every pixel when P > 0 (empty tiles get the background), so only the
    # P == 0 case needs the reference's zero fill (rasterize_points.cu:69-73)
    alloc = torch.zeros if P == 0 else torch.empty
    out_color = alloc((NUM_CHANNELS, H, W), **fopts)
    out_invdepth = alloc((1, H, W), **fopts)
    radii = alloc((P,), dtype=torch.int32, device=dev)  # (preprocess writes every Gaussian's radius)
    geom, binning, img = _Resizer(dev), _Resizer(dev), _Resizer(dev)
    rendered = 0
    if P != 0:
        if dev.type != "cuda":
            raise RuntimeError("rasterize_gaussians needs tensors on a HIP (cuda) device; "
                               "there is no CPU implementation")
        L = _lib.load()
        M = int(sh.size(1)) if (sh is not None and sh.numel() != 0 and sh.size(0) != 0) else 0
        means3D = _dev_f32(means3D, dev, "means3D")
        colors = _dev_f32(colors, dev, "colors_precomp")
        if colors is not None and colors.numel() and colors.data_ptr() % 16:
            colors = colors.clone()
        opacity = _dev_f32(opacity, dev, "opacities")
        scales = _dev_f32(scales, dev, "scales")
        rotations = _dev_f32(rotations, dev, "rotations")
        cov3D_precomp = _dev_f32(cov3D_precomp, dev, "cov3D_precomp")
        background = _dev_f32(background, dev, "bg")
        viewmatrix = _dev_f32(viewmatrix, dev, "viewmatrix")
        projmatrix = _dev_f32(projmatrix, dev, "projmatrix")
        args = (geom.cb, binning.cb, img.cb, None, P, int(degree), M, _ptr(background), W, H,
                _ptr(means3D), _ptr(sh), _ptr(colors), _ptr(opacity), _ptr(scales),
                float(scale_modifier), _ptr(rotations), _ptr(cov3D_precomp), _ptr(viewmatrix),
                _ptr(projmatrix), _ptr(campos), float(tan_fovx), float(tan_fovy),
                int(bool(prefiltered)), out_color.data_ptr(), out_invdepth.data_ptr(),
                int(bool(antialiasing)), radii.data_ptr(), int(bool(debug)))
        bound = L.gsr_forward_async_bound(P, W, H)
        with torch.cuda.device(dev):
            if (not debug and not exact_binning and bound < 0x7FFFFFFF
                    and L.gsr_binning_bytes(bound) <= ASYNC_BINNING_MB << 20):
                ring = _RINGS.get(dev)
                if ring is None:
                    ring = _RINGS[dev] = _StatusRing()
                status, ev, k = ring.take(dev)
                _lib.check(L.gsr_forward_async(*args, status.data_ptr(), int(numerics), _stream(dev)),
                           "rasterize_gaussians")
                ev.record(torch.cuda.current_stream(dev))
                rendered = PendingCount(status, ev)
                ring.bind(k, ev, rendered)
            else:
                rendered = _lib.check(L.gsr_forward_ex(*args, int(numerics), _stream(dev)), "rasterize_gaussians")
    return rendered, out_color, radii, geom.t, binning.t, img.t, out_invdepth


class _Scratch:
    """The three scratch arenas of inference forwards on one (device, stream), kept between calls
    (stream order makes the reuse safe) and handed to the C ABI through its preallocated-scratch
    resizers (include/gsr.h gsr_scratch_*): no host callback and no allocation per call."""

    def __init__(self, device):
        self.device = device
        self.bufs = [torch.empty((0,), dtype=torch.uint8, device=device) for _ in range(3)]
        self.s = _lib.Scratch()
        self.sizes = {}
        self._last = None

    def fit(self, L, P, W, H, bound):
        key = (P, W, H)
        if key == self._last:  # the same shape as the previous call: the struct is current
            return self.s
        self._last = key
        need = self.sizes.get(key)
        if need is None:
            need = self.sizes[key] = (L.gsr_geometry_bytes(P, W, H), L.gsr_binning_bytes(bound),
                                      L.gsr_image_bytes(W, H))
        for i, n in enumerate(need):
            if self.bufs[i].numel() < n:
                self.bufs[i] = torch.empty((int(n),), dtype=torch.uint8, device=self.device)
        s = self.s
        s.geometry, s.geometry_cap = self.bufs[0].data_ptr(), self.bufs[0].numel()
        s.binning, s.binning_cap = self.bufs[1].data_ptr(), self.bufs[1].numel()
        s.image, s.image_cap = self.bufs[2].data_ptr(), self.bufs[2].numel()
        return s


_SCRATCH = collections.OrderedDict()  # (device, stream handle) -> _Scratch, least recently used first
_SCRATCH_MAX = 8
_SCRATCH_FNS = None
_BOUNDS = {}  # (P, W, H) -> the async bound when the no-sync forward applies, else None


def clear_scratch():
    """Release the inference scratch arenas kept per (device, stream) (they are re-created on the
    next call).  At most _SCRATCH_MAX streams keep arenas; the least recently used is dropped first.
    A stream handle that the runtime reuses after its stream was destroyed inherits that stream's
    arenas, which is safe: they are scratch, used in stream order."""
    _SCRATCH.clear()


def rasterize_inference(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                        viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, antialiasing,
                        numerics=None):
    """The forward of an inference call (no gradient, debug and prefiltered off): the images of
    rasterize_gaussians -- (color[32,H,W], radii[P], invdepth[1,H,W]), bit-identical -- without its
    per-call host work: the scratch arenas are kept per (device, stream) and passed preallocated
    (no allocator callbacks), no status copy (no error is possible without prefiltered), and no
    autograd node.  Returns None when it does not apply (the caller takes rasterize_gaussians)."""
    global _SCRATCH_FNS
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    P, H, W = int(means3D.size(0)), int(image_height), int(image_width)
    dev = means3D.device
    if P == 0 or dev.type != "cuda" or colors is None or colors.numel() == 0:
        return None
    dix = means3D.get_device()
    if dix != torch._C._cuda_getDevice():
        # the library sizes its persistent grids and raises LDS limits on the current device: the
        # general path enters the inputs' device first (no device switch on this hot path)
        return None
    L = _lib.load()
    bound = _BOUNDS.get((P, W, H), 0)
    if bound == 0:
        bound = L.gsr_forward_async_bound(P, W, H)
        if bound >= 0x7FFFFFFF or L.gsr_binning_bytes(bound) > ASYNC_BINNING_MB << 20:
            bound = None
        _BOUNDS[(P, W, H)] = bound
    if bound is None:
        return None
    if numerics is None:
        numerics = DEFAULT_NUMERICS
    ts = [background, means3D, colors, opacity, scales, rotations, viewmatrix, projmatrix]
    f32 = torch.float32
    for i, t_ in enumerate(ts):  # (one pass: device / dtype check and contiguous rows)
        if t_ is not None and t_.numel():
            if t_.get_device() != dix or t_.dtype is not f32:
                return None  # (the general path raises the reference's errors)
            ts[i] = t_.contiguous()
    background, means3D, colors, opacity, scales, rotations, viewmatrix, projmatrix = ts
    if colors.data_ptr() % 16:
        colors = colors.clone()
    cov = cov3D_precomp if (cov3D_precomp is not None and cov3D_precomp.numel()) else None
    if cov is not None:
        if cov.device != dev or cov.dtype != torch.float32:
            return None
        cov = cov.contiguous()
    stream = torch._C._cuda_getCurrentRawStream(dix)  # (the handle; torch.cuda.current_stream builds an object)
    key = (dix, stream)
    sc = _SCRATCH.get(key)
    if sc is None:
        sc = _SCRATCH[key] = _Scratch(dev)
        while len(_SCRATCH) > _SCRATCH_MAX:
            _SCRATCH.popitem(last=False)
    else:
        _SCRATCH.move_to_end(key)
    s = sc.fit(L, P, W, H, bound)
    if _SCRATCH_FNS is None:
        addr = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
        _SCRATCH_FNS = tuple(_lib.ALLOC_FN(addr(f)) for f in (L.gsr_scratch_geometry, L.gsr_scratch_binning,
                                                                L.gsr_scratch_image))
    fopts = dict(dtype=torch.float32, device=dev)
    out_color = torch.empty((NUM_CHANNELS, H, W), **fopts)
    out_invdepth = torch.empty((1, H, W), **fopts)
    radii = torch.empty((P,), dtype=torch.int32, device=dev)
    _lib.check(L.gsr_forward_async(*_SCRATCH_FNS, ctypes.addressof(s), P, 0, 0, _ptr(background), W, H,
                                   means3D.data_ptr(), None, colors.data_ptr(), _ptr(opacity), _ptr(scales),
                                   float(scale_modifier), _ptr(rotations), _ptr(cov), _ptr(viewmatrix),
                                   _ptr(projmatrix), None, float(tan_fovx), float(tan_fovy), 0,
                                   out_color.data_ptr(), out_invdepth.data_ptr(), int(bool(antialiasing)),
                                   radii.data_ptr(), 0, None, int(numerics), stream),
               "rasterize_gaussians")
    return out_color, radii, out_invdepth


def rasterize_gaussians_backward(background, means3D, radii, colors, opacities, scales, rotations,
                                 scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx,
                                 tan_fovy, dL_dout_color, dL_dout_invdepth, sh, degree, campos,
                                 geomBuffer, R, binningBuffer, imageBuffer, antialiasing, debug, *, numerics=None):
    """RasterizeGaussiansBackwardCUDA (rasterize_points.cu:127-223).  Returns
    (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations).
    numerics: as rasterize_gaussians."""
    if numerics is None:
        numerics = DEFAULT_NUMERICS
    P = int(means3D.size(0))
    H = int(dL_dout_color.size(1))
    W = int(dL_dout_color.size(2))
    M = int(sh.size(1)) if (sh is not None and sh.numel() != 0 and sh.size(0) != 0) else 0
    dev = means3D.device
    o = dict(dtype=torch.float32, device=dev)
    dL_dmeans3D = torch.zeros((P, 3), **o)
    dL_dmeans2D = torch.zeros((P, 3), **o)
    dL_dcolors = torch.zeros((P, NUM_CHANNELS), **o)
    dL_dconic = torch.zeros((P, 2, 2), **o)
    dL_dopacity = torch.zeros((P, 1), **o)
    dL_dcov3D = torch.zeros((P, 6), **o)
    dL_dsh = torch.zeros((P, M, 3), **o)
    dL_dscales = torch.zeros((P, 3), **o)
    dL_drotations = torch.zeros((P, 4), **o)
    dL_dinvdepths = torch.zeros((0, 1), **o)
    inv_pix = None
    if dL_dout_invdepth is not None and dL_dout_invdepth.numel() != 0 and dL_dout_invdepth.size(0) != 0:
        dL_dinvdepths = torch.zeros((P, 1), **o)
        inv_pix = _dev_f32(dL_dout_invdepth, dev, "dL_dout_invdepth")
    if P != 0:
        L = _lib.load()
        dL_dout_color = _dev_f32(dL_dout_color, dev, "dL_dout_color")
        colors = _dev_f32(colors, dev, "colors_precomp")
        if colors is not None and colors.numel() and colors.data_ptr() % 16:
            colors = colors.clone()
        means3D = _dev_f32(means3D, dev, "means3D")
        opacities = _dev_f32(opacities, dev, "opacities")
        scales = _dev_f32(scales, dev, "scales")
        rotations = _dev_f32(rotations, dev, "rotations")
        cov3D_precomp = _dev_f32(cov3D_precomp, dev, "cov3D_precomp")
        background = _dev_f32(background, dev, "bg")
        viewmatrix = _dev_f32(viewmatrix, dev, "viewmatrix")
        projmatrix = _dev_f32(projmatrix, dev, "projmatrix")
        with torch.cuda.device(dev):
            rc = L.gsr_backward_ex(
                P, int(degree), M, int(R), _ptr(background), W, H, _ptr(means3D), _ptr(sh),
                _ptr(colors), _ptr(opacities), _ptr(scales), float(scale_modifier), _ptr(rotations),
                _ptr(cov3D_precomp), _ptr(viewmatrix), _ptr(projmatrix), _ptr(campos),
                float(tan_fovx), float(tan_fovy), _ptr(radii), _ptr(geomBuffer), _ptr(binningBuffer),
                _ptr(imageBuffer), dL_dout_color.data_ptr(), _ptr(inv_pix), dL_dmeans2D.data_ptr(),
                dL_dconic.data_ptr(), dL_dopacity.data_ptr(), dL_dcolors.data_ptr(),
                _ptr(dL_dinvdepths), dL_dmeans3D.data_ptr(), dL_dcov3D.data_ptr(), _ptr(dL_dsh),
                dL_dscales.data_ptr(), dL_drotations.data_ptr(), int(bool(antialiasing)),
                int(bool(debug)), int(numerics), _stream(dev))
        _lib.check(rc, "rasterize_gaussians_backward")
    return (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
            dL_drotations)


def mark_visible(means3D, viewmatrix, projmatrix):
    """markVisible (rasterize_points.cu:225-244): bool[P], view-space z > 0.2."""
    P = int(means3D.size(0))
    dev = means3D.device
    present = torch.zeros((P,), dtype=torch.bool, device=dev)
    if P != 0:
        L = _lib.load()
        means3D = _dev_f32(means3D, dev, "means3D")
        viewmatrix = _dev_f32(viewmatrix, dev, "viewmatrix")
        projmatrix = _dev_f32(projmatrix, dev, "projmatrix")
        with torch.cuda.device(dev):
            rc = L.gsr_mark_visible(P, means3D.data_ptr(), viewmatrix.data_ptr(),
                                    projmatrix.data_ptr(), present.data_ptr(), _stream(dev))
        _lib.check(rc, "mark_visible")
    return present
