"""World-size-2 run of the REAL rasterizer (frame sharding + all-gather of the rendered frames), two
ranks on one GPU over gloo (the 8-GPU RCCL run is the driver's; the collective calls are the same,
parallel.gather_frames).  The gathered batch must equal a single-process render of all frames,
bit for bit (frames are independent; each rank runs the batched entry on its shard)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
N_FRAMES, P, W = 5, 20000, 128


def _inputs(frames):
    from guava_renderer_amd import scenes
    sc = scenes.avatar_cloud(P, seed=9)
    cams = [scenes.frame_cameras(N_FRAMES, W, W, seed=1000)[i] for i in frames]
    dev = torch.device("cuda:0")
    t = lambda x: torch.tensor(np.ascontiguousarray(x), device=dev)  # noqa: E731
    args = [t(sc[k]) for k in ("means3D", "colors", "opacities", "scales", "rotations")]
    views = t(np.stack([c["viewmatrix"].reshape(16) for c in cams]))
    projs = t(np.stack([c["projmatrix"].reshape(16) for c in cams]))
    tanf = t(np.array([[c["tanfovx"], c["tanfovy"]] for c in cams], np.float32))
    return args, views, projs, tanf, torch.zeros((len(frames), 32), device=dev)


def _render(frames):
    from guava_renderer_amd.batch import BatchRasterizer
    args, views, projs, tanf, bg = _inputs(frames)
    r = BatchRasterizer(len(frames), P, W, W, R_capacity=16 * P * len(frames), device="cuda:0")
    col, _, _ = r.forward(*args, views, projs, tanf, bg)
    r.poll(wait=True)
    return col.clone()


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from guava_renderer_amd import parallel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = parallel.shard_range(N_FRAMES, rank, world)
        local = _render(list(range(lo, hi)))
        full = parallel.gather_frames(local.cpu(), N_FRAMES)
        # the 8-bit exchange bench.py runs at N>1: encoded on the GPU, gathered as uint8
        full8 = parallel.gather_frames(parallel.frames_to8b(local).cpu(), N_FRAMES)
        if rank == 0:
            q.put((full.numpy(), full8.numpy()))
    finally:
        dist.destroy_process_group()


def test_two_ranks_real_rasterizer_gather():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, gathered8 = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = _render(list(range(N_FRAMES))).cpu().numpy()
    assert gathered.shape == ref.shape
    np.testing.assert_array_equal(gathered, ref)
    np.testing.assert_array_equal(gathered8, _to8b(ref[:, :3]))


def _to8b(img):
    """GUAVA's to8b (utils/general_utils.py:316-317)."""
    return (255 * np.clip(img, 0, 1)).astype(np.uint8)


def test_frames_to8b_matches_to8b():
    from guava_renderer_amd import parallel
    rng = np.random.default_rng(3)
    x = rng.uniform(-0.5, 1.5, (3, 32, 37, 53)).astype(np.float32)  # ragged plane: the scalar kernel
    x[0, 0, 0, :5] = [0.0, 1.0, 1.0 / 255, 254.999 / 255, 0.5]
    for shape in ((3, 32, 37, 53), (2, 32, 64, 64)):
        xs = np.ascontiguousarray(x[:shape[0], :, :shape[2], :shape[3]]) if shape[2] <= 37 else \
            rng.uniform(-0.5, 1.5, shape).astype(np.float32)
        got = parallel.frames_to8b(torch.tensor(xs, device="cuda:0")).cpu().numpy()
        np.testing.assert_array_equal(got, _to8b(xs[:, :3]))


def _nccl_worker(port, q):
    """World-1 RCCL group on the one GPU: FrameGather's device path (async RCCL work on the PG's own
    stream, staging buffers reused every other batch) on real renders, each gathered batch checked after the
    next batch was pushed (so the overlap is exercised)."""
    import torch.distributed as dist
    from guava_renderer_amd import parallel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        batches = [[0, 1], [2, 3], [4, 0], [1, 2]]
        refs = [_render(b)[:, :3].clone() for b in batches]
        fg = parallel.FrameGather(2, (3, W, W), torch.float32, dev)
        ok = True
        prev = None
        for b, ref in zip(batches, refs):
            fg.push(_render(b)[:, :3])
            if prev is not None:  # the previous batch's buffer, read while this one is in flight
                pb, pref = prev
                fg.work[pb].wait()  # this stream after that batch's exchange
                ok = ok and torch.equal(fg.bufs[pb][1], pref)
            prev = ((fg.k - 1) % len(fg.bufs), ref)
        last = fg.wait()
        ok = ok and torch.equal(last, refs[-1])
        # uint8 staging: the 32-channel frames are encoded (to8b) into the buffer the collective sends
        f8 = parallel.FrameGather(2, (3, W, W), torch.uint8, dev)
        for b in batches:
            f8.push(_render(b))
        ok = ok and torch.equal(f8.wait(), parallel.frames_to8b(_render(batches[-1])))
        q.put(bool(ok))
    finally:
        dist.destroy_process_group()


def test_frame_gather_device_path_rccl_world1():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(port, q))
    p.start()
    ok = q.get(timeout=240)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert ok
