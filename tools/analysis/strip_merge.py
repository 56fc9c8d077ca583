"""How much a tile-level merge of render_bwd's per-strip atomics could save: on one C2 frame (the
quad_tail.py scene, GPU forward through the drop-in call), the strip survivors (set strip bits over
the tile lists) against the list entries with at least one -- render_bwd writes one 160-B atomic row
set per strip survivor; a merge of a tile's four strips would write one per such entry.
python tools/analysis/strip_merge.py  (GPU)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from guava_renderer_amd import scenes  # noqa: E402
from helpers import gpu_forward  # noqa: E402

d = scenes.avatar_cloud(100000, seed=0)
cam = scenes.frame_cameras(2, 512, 512, seed=1000)[1]
d.update(cam)
d["bg"] = np.zeros(32, np.float32)
_, _, _, st = gpu_forward(d)
R = int(st["R"])
sm = st["smask"][:R].astype(np.int64)
bits = sum((sm >> s) & 1 for s in range(4))
print(f"list entries {R}, with a strip survivor {int((sm != 0).sum())}, strip survivors {int(bits.sum())}, "
      f"survivors per reaching entry {bits.sum() / max((sm != 0).sum(), 1):.3f}")
