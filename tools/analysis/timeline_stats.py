"""Summarise gpurun_out/timeline.npz (tools/timeline.py)."""
import sys

import numpy as np

z = np.load(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/timeline.npz")
tl = z["tl"].astype(np.int64)
valid = tl[:, 1] != 0
r = tl[valid]
st = r[:, 0].astype(np.uint32).astype(np.int64)
en = r[:, 1].astype(np.uint32).astype(np.int64)
ks = r[:, 2]
t0 = st.min()
st -= t0
en -= t0
dur = en - st
T = en.max()
print(f"items {len(r)} span {T / 100:.1f} us  mean dur {dur.mean() / 100:.1f} us  max {dur.max() / 100:.1f} us")
o = np.argsort(-dur)[:8]
idx = np.nonzero(valid)[0]
for i in o:
    print(f"  item {idx[i]:6d} start {st[i] / 100:7.1f} end {en[i] / 100:7.1f} dur {dur[i] / 100:7.1f} us "
          f"ksteps {ks[i]:5d}  ns/kstep {dur[i] * 10 / max(ks[i], 1):6.0f}")
bins = np.linspace(0, T, 11)
for a, b in zip(bins[:-1], bins[1:]):
    print(f"  {a / 100:7.1f}-{b / 100:7.1f} us: items running at bin end {((st < b) & (en >= b)).sum():5d}, "
          f"k-steps done in bin {int((ks * np.clip((np.minimum(en, b) - np.maximum(st, a)) / np.maximum(dur, 1), 0, 1)).sum())}")
