"""Render work counters (gsr_render_counters: k-steps, pairs blended / contributing, entries
staged) of one B-frame avatar batch of the bench workload (python tools/render_stats.py [B])."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from guava_renderer_amd.batch import render_counters  # noqa: E402


class A:
    pipeline = "avatar"
    config = "c2"
    inflight = 1
    refine = False


B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
dev = torch.device("cuda:0")
w = bench.Workload(A, bench._workload("c2"), B, 0, B, dev, 0)
w.step_on(0)
torch.cuda.synchronize()
c = render_counters(lambda: w.step_on(0))
print(f"B={B}", c, flush=True)
