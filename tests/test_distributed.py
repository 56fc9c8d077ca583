"""World-size-2 gloo tests of the frame-sharded multi-GPU path (guava_renderer_amd/parallel.py).

The rasterization itself is replaced here by a deterministic per-frame function (no GPU); what is
tested is the sharding, ordering and the two consumer-side collectives bench.py and a trainer use.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from guava_renderer_amd import parallel


def test_shard_range_covers_exactly_once():
    for n in (0, 1, 5, 8, 31, 32, 33):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                lo, hi = parallel.shard_range(n, r, world)
                assert 0 <= lo <= hi <= n
                seen.extend(range(lo, hi))
            assert seen == list(range(n))
    with pytest.raises(ValueError):
        parallel.shard_range(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_render(frame_ids):
    # stands in for one frame of a rasterizer output [C=32, 4, 4]
    f = torch.as_tensor(frame_ids, dtype=torch.float32).view(-1, 1, 1, 1)
    return f * 1000 + torch.arange(32 * 16, dtype=torch.float32).view(1, 32, 4, 4)


def _worker(rank, world, port, n_frames, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frames = parallel.shard_frames(list(range(n_frames)))
        local = _fake_render(frames) if frames else torch.zeros((0, 32, 4, 4))
        full = parallel.gather_frames(local, n_frames)
        ok_gather = torch.equal(full, _fake_render(list(range(n_frames))))
        g = {"colors": torch.full((10, 32), float(rank + 1)), "opacity": torch.full((10, 1), 2.0 * rank),
             "none": None}
        parallel.reduce_shared_grads(g)
        ok_reduce = (torch.all(g["colors"] == sum(r + 1 for r in range(world))).item()
                     and torch.all(g["opacity"] == sum(2.0 * r for r in range(world))).item())
        ok_stream = True
        if n_frames % world == 0:  # FrameGather (bench.py's overlapped exchange): equal shards
            fg = parallel.FrameGather(len(frames), (32, 4, 4), torch.float32, torch.device("cpu"))
            for step in range(3):  # successive batches through the two staging buffers
                ids = [step * n_frames + f for f in frames]
                fg.push(_fake_render(ids))
                got = fg.wait()
                want = _fake_render([step * n_frames + f for f in range(n_frames)])
                ok_stream = ok_stream and torch.equal(got, want)
            # the 8-bit exchange (bench.py's default at N>1): uint8 frames as the consumer writes them
            f8 = parallel.FrameGather(len(frames), (3, 4, 4), torch.uint8, torch.device("cpu"))
            for step in range(3):
                ids = [step * n_frames + f for f in frames]
                f8.push((_fake_render(ids)[:, :3] % 251).to(torch.uint8))
                got = f8.wait()
                want = (_fake_render([step * n_frames + f for f in range(n_frames)])[:, :3] % 251).to(torch.uint8)
                ok_stream = ok_stream and got.dtype == torch.uint8 and torch.equal(got, want)
            # float32 frames into the uint8 exchange on the host: to8b (general_utils.py:316-317)
            for step in range(2):
                ids = [step * n_frames + f for f in frames]
                fr = _fake_render(ids)[:, :5] / 700.0 - 0.2
                f8.push(fr)
                got = f8.wait()
                full_fr = _fake_render([step * n_frames + f for f in range(n_frames)])[:, :3] / 700.0 - 0.2
                want = torch.from_numpy((255 * np.clip(full_fr.numpy(), 0, 1)).astype(np.uint8))
                ok_stream = ok_stream and torch.equal(got, want)
        q.put((rank, ok_gather, ok_reduce and ok_stream))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_frames", [8, 5, 1])
def test_gather_and_reduce_world2(n_frames):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_frames, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(r[0] for r in res) == [0, 1]
    assert all(r[1] and r[2] for r in res), res


def test_stream_budget_leaves_a_queue_for_rccl(monkeypatch):
    """At N > 1 the bench keeps at most GPU_MAX_HW_QUEUES - 1 compute streams (RCCL runs every
    collective on ProcessGroupNCCL's internal stream, FrameGather adds none), so the exchange never
    shares a hardware queue with a persistent render kernel; at N = 1 all queues compute."""
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    assert parallel.stream_budget(4, 1) == 4
    assert parallel.stream_budget(4, 2) == 3
    assert parallel.stream_budget(4, 8) == 3
    assert parallel.stream_budget(2, 8) == 2
    assert parallel.stream_budget(1, 8) == 1
    assert parallel.stream_budget(4, 2, hw_queues=8) == 4
    import inspect
    src = inspect.getsource(parallel.FrameGather)
    assert "torch.cuda.Stream(" not in src  # no side stream of its own
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    bench_src = open(os.path.join(root, "bench.py")).read()
    assert "a.inflight = parallel.stream_budget(a.inflight, world)" in bench_src


def test_bench_rank_launch_contract(monkeypatch):
    """bench.py --gpus N starts its own N ranks (torch.distributed.run as a child process, rendezvous
    on 127.0.0.1) when no launcher set WORLD_SIZE, and refuses a launcher world that differs from N."""
    import subprocess
    import sys as _sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1")
    r = subprocess.run([_sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr
    _sys.path.insert(0, root)
    import bench
    seen = {}

    class Done:
        returncode = 0

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return Done()
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.setattr(_sys, "argv", ["bench.py", "--gpus", "4", "--steps", "7"])
    assert bench._launch_ranks(4) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-4:] == ["--gpus", "4", "--steps", "7"]
