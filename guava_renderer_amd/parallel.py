"""Frame sharding across GPUs (one process per GPU).

Frames (camera views / poses of an avatar) are independent units of the rasterizer: each rank
renders its own contiguous slice of the frame list with no collective on the data path
(bench.py reports "scaling": "weak").  The only exchange is at the consumer boundary:
`gather_frames` assembles the full [N, ...] batch on every rank (all_gather over RCCL on
GPUs, gloo in the CPU tests), and `reduce_shared_grads` sums per-frame gradients of a
shared avatar (the DP gradient all-reduce a trainer would do; one flat bucket, since xGMI
rings are per-link bound and favour few large messages).
"""
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
