"""Frame sharding across GPUs (one process per GPU).

Frames (camera views / poses of an avatar) are independent units of the rasterizer: each rank
renders its own contiguous slice of the frame list with no collective on the data path
(bench.py reports "scaling": "weak").  The only exchange is at the consumer boundary:
`gather_frames` assembles the full [N, ...] batch on every rank (all_gather over RCCL on
GPUs, gloo in the CPU tests), `FrameGather` does the same for a stream of equal batches without
copies and overlapped with the next batch's rendering, and `reduce_shared_grads` sums per-frame
gradients of a
shared avatar (the DP gradient all-reduce a trainer would do; one flat bucket, since xGMI
rings are per-link bound and favour few large messages).
"""
import ctypes
import os

import torch
import torch.distributed as dist


def shard_range(n_frames, rank, world):
    """Contiguous [lo, hi) slice of `n_frames` for `rank`; the first n % world ranks get one
    extra frame, so ragged counts are covered exactly once."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(int(n_frames), world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard_frames(items, rank=None, world=None):
    """Rank-local slice of a per-frame sequence or tensor (leading dim = frame)."""
    rank = dist.get_rank() if rank is None else rank
    world = dist.get_world_size() if world is None else world
    lo, hi = shard_range(len(items), rank, world)
    return items[lo:hi]


def gather_frames(local, n_frames, group=None):
    """All-gather rank-local frames [n_local, ...] into the full [n_frames, ...] batch, in
    frame order.  Ragged shards are padded to the largest shard for the collective."""
    world = dist.get_world_size(group)
    counts = [shard_range(n_frames, r, world) for r in range(world)]
    cap = max(hi - lo for lo, hi in counts)
    pad = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    out = torch.empty((world * cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    parts = [out[r * cap: r * cap + (hi - lo)] for r, (lo, hi) in enumerate(counts)]
    return torch.cat(parts, 0)


def frames_to8b(frames, channels=3, out=None):
    """GUAVA's to8b (utils/general_utils.py:316-317: (255 * clip(x, 0, 1)).astype(uint8), applied to
    every rendered frame at main/test.py:85) of the first `channels` planes of [B, C, H, W] float32
    device frames -> [B, channels, H, W] uint8, one HIP pass (gsr_frames_to8b).  The exchange then
    carries 3 bytes per pixel instead of 12."""
    from . import _lib
    if frames.device.type != "cuda" or frames.dtype != torch.float32 or frames.dim() != 4:
        raise ValueError("frames_to8b: needs [B,C,H,W] float32 frames on a HIP device")
    B, Cs, H, W = frames.shape
    if channels > Cs or frames.stride(3) != 1 or frames.stride(2) != W or frames.stride(1) != H * W:
        raise ValueError("frames_to8b: frames must be dense [B,C,H,W] planes with C >= channels")
    if out is None:
        out = torch.empty((B, channels, H, W), dtype=torch.uint8, device=frames.device)
    elif tuple(out.shape) != (B, channels, H, W) or out.dtype != torch.uint8 or not out.is_contiguous():
        raise ValueError("frames_to8b: out must be a contiguous [B,channels,H,W] uint8 tensor")
    st = ctypes.c_void_p(torch.cuda.current_stream(frames.device).cuda_stream)
    _lib.check(_lib.load().gsr_frames_to8b(B, channels, H, W, frames.data_ptr(), frames.stride(0),
                                           out.data_ptr(), st), "gsr_frames_to8b")
    return out


def to8b_host(frames, channels):
    """Host to8b of the first `channels` planes of [B, C, H, W] frames (utils/general_utils.py:316-317:
    (255 * clip(x, 0, 1)).astype(uint8), truncation toward zero, NaN -> 0 as frames_to8b)."""
    x = torch.nan_to_num(frames[:, :channels].float(), nan=0.0).clamp_(0.0, 1.0)
    return (x * 255.0).to(torch.uint8)


def stream_budget(inflight, world, hw_queues=None):
    """Compute streams the bench may keep busy: GPU_MAX_HW_QUEUES hardware queues per process (4 on
    the box, HIP's default); at N > 1 one of them is left to the collective (ProcessGroupNCCL runs
    every RCCL call on its own internal stream), so the all-gather never queues behind a persistent
    render kernel on a shared hardware queue."""
    if hw_queues is None:
        hw_queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
    reserved = 1 if world > 1 else 0
    return max(1, min(int(inflight), hw_queues - reserved))


class FrameGather:
    """Overlapped all-gather of a stream of equal per-rank batches [n_local, *shape] into
    [world * n_local, *shape] on every rank (frame order = rank order, as shard_range's contiguous
    slices).  `push(frames)` writes the rank's frames into a staging buffer on the current stream
    and issues the collective asynchronously: RCCL runs it on ProcessGroupNCCL's internal stream once
    the staging write is done (no side stream of our own: with GPU_MAX_HW_QUEUES = 4 the bench keeps
    3 compute streams + that one, `stream_budget`), so batch i's exchange runs under batch i+1's
    rendering; `n_buffers` batches may be in flight (a push orders its stream after the exchange
    that last used its buffer).  `wait()` orders the current stream after every exchange pushed so
    far and returns the latest gathered batch.  One collective per batch, no padding and no
    concatenation (RCCL rings over xGMI are per-link bound: one large message per batch).
    With dtype uint8 and float32 [n_local, C, H, W] frames, push() encodes the first shape[0]
    planes as to8b: frames_to8b straight into the staging buffer when both are on the same HIP
    device, the host form (to8b_host) otherwise (the consumer's 8-bit frames, 4x fewer bytes on the
    links than f32)."""

    def __init__(self, n_local, shape, dtype, device, group=None, n_buffers=2):
        self.group = group
        self.world = dist.get_world_size(group)
        self.device = device
        self.bufs = [(torch.empty((n_local,) + tuple(shape), dtype=dtype, device=device),
                      torch.empty((self.world * n_local,) + tuple(shape), dtype=dtype, device=device))
                     for _ in range(n_buffers)]
        self.work = [None] * n_buffers
        self.k = 0
        self.last = None

    def _stage(self, src, frames):
        if src.dtype == torch.uint8 and frames.dtype == torch.float32:
            if frames.is_cuda and src.is_cuda and frames.device == src.device:
                frames_to8b(frames, src.shape[1], out=src)
            else:
                src.copy_(to8b_host(frames, src.shape[1]))
        else:
            src.copy_(frames)

    def push(self, frames):
        j = self.k % len(self.bufs)
        self.k += 1
        src, dst = self.bufs[j]
        if self.device.type != "cuda":  # CPU (gloo): synchronous
            self._stage(src, frames)
            dist.all_gather_into_tensor(dst, src, group=self.group)
            self.last = dst
            return
        if self.work[j] is not None:
            self.work[j].wait()  # the current stream waits for the exchange that last read src / wrote dst
        self._stage(src, frames)
        self.work[j] = dist.all_gather_into_tensor(dst, src, group=self.group, async_op=True)
        self.last = dst

    def wait(self):
        for wk in self.work:
            if wk is not None:
                wk.wait()
        return self.last


def reduce_shared_grads(grads, group=None):
    """Sum a dict of per-rank gradient tensors of shared (stride-0) avatar attributes over ranks,
    in place, as one flattened bucket."""
    keys = [k for k in sorted(grads) if grads[k] is not None]
    if not keys:
        return grads
    flat = torch.cat([grads[k].reshape(-1) for k in keys])
    dist.all_reduce(flat, group=group)
    off = 0
    for k in keys:
        n = grads[k].numel()
        grads[k].copy_(flat[off: off + n].view_as(grads[k]))
        off += n
    return grads


def cu_masks(n_cus, prep_cus, mode="spread"):
    """(prep mask, render mask) as lists of 32-bit words over n_cus CUs: the prep slice takes
    prep_cus CUs -- CU i * step + (i mod 8) for step = n_cus / prep_cus ("spread": one share on each
    XCD whether the mask's bit order interleaves the 8 XCDs or runs through them one after the
    other) or the first prep_cus ("lo") -- and the render slice the rest.  prep_cus == 0: both masks
    are every CU."""
    n_words = (n_cus + 31) // 32
    prep = [0] * n_words
    if prep_cus <= 0:
        full = [0] * n_words
        for c in range(n_cus):
            full[c // 32] |= 1 << (c % 32)
        return full, list(full)
    if not 0 < prep_cus < n_cus:
        raise ValueError(f"prep_cus must be in (0, {n_cus})")
    if mode == "spread":
        blk = max(1, n_cus // 8)
        chosen = set()
        for t in range(prep_cus):  # share t: block t mod 8, residue mod 8 rotating with the block
            b, w = t % 8, t // 8
            c = b * blk + (w * 8 + b + w // max(1, blk // 8)) % blk
            while c in chosen:
                c = (c + 1) % n_cus
            chosen.add(c)
    elif mode == "lo":
        chosen = set(range(prep_cus))
    else:
        raise ValueError(f"unknown mode {mode!r}")
    render = [0] * n_words
    for c in range(n_cus):
        if c in chosen:
            prep[c // 32] |= 1 << (c % 32)
        else:
            render[c // 32] |= 1 << (c % 32)
    return prep, render


class SplitPlacement:
    """Batches in flight with the compositing kernel on its own CU slice (include/gsr.h
    gsr_stream_create_cu_mask / gsr_set_render_stream): `n_prep` streams for the deform + binning
    chains of the batches, each routed so its forwards' render kernels run on ONE shared render
    stream.  prep_cus > 0 masks the prep streams to that many CUs and the render stream to the rest
    (the persistent render grid is sized to them); prep_cus == 0 keeps every stream on every CU (the
    routing alone).  `streams` are torch ExternalStreams of the prep streams (use with
    torch.cuda.stream); close() destroys them."""

    def __init__(self, n_prep, prep_cus, device, mode="spread"):
        self.mode = mode
        from . import _lib
        L = self.L = _lib.load()
        n_cus = torch.cuda.get_device_properties(device).multi_processor_count
        pm, rm = cu_masks(n_cus, prep_cus, mode)
        self.handles = []

        def make(mask):
            arr = (ctypes.c_uint32 * len(mask))(*mask)
            h = ctypes.c_void_p()
            _lib.check(L.gsr_stream_create_cu_mask(len(mask), arr, ctypes.byref(h)), "gsr_stream_create_cu_mask")
            self.handles.append(h.value)
            return h.value
        self.render_handle = make(rm)
        self.prep_handles = [make(pm) for _ in range(n_prep)]
        for h in self.prep_handles:
            _lib.check(L.gsr_set_render_stream(h, self.render_handle), "gsr_set_render_stream")
        self.streams = [torch.cuda.ExternalStream(h, device=device) for h in self.prep_handles]
        self.render_stream = torch.cuda.ExternalStream(self.render_handle, device=device)
        self.prep_cus, self.render_cus = sum(bin(w).count("1") for w in pm), sum(bin(w).count("1") for w in rm)

    def close(self):
        torch.cuda.synchronize()
        for h in self.handles:
            self.L.gsr_stream_destroy(h)
        self.handles = []
