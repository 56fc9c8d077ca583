"""CPU baselines of SURVEY.md 8(d) / BASELINE.md (the reference has no CPU path of its own):

* the CPU oracle (oracle/gsr_oracle.c, a line-cited C restatement of the reference rasterizer) on
  config 1 (10k random Gaussians, 256 x 256, canonical camera): projection + binning + stable sort
  (forward.cu:151-269, rasterizer_impl.cu:70-138,306-311) and the full forward render, at 1 thread
  and at every core this process may run on (os.sched_getaffinity); 3 warm-ups, median of 20;
* the full forward on config 2 (the 100k avatar cloud, 512 x 512) at every core, median of 5;
* in the build container only (it needs /root/reference): the reference's own torch-CPU
  `lbs_wobeta` (models/modules/flame/lbs.py:255-333) at V = 10,595, J = 55, B = 1 and B = 32 with
  8 torch threads, median of 10.

    python tools/cpu_baselines.py [out.json]

TEST/MEASUREMENT INFRASTRUCTURE: uses oracle/ as the thing timed (cpu_baseline, kind "port").
"""
import importlib.util
import json
import os
import platform
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def _median_time(fn, warm, reps):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def _cpu_model():
    try:
        return next(ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name"))
    except (OSError, StopIteration):
        return platform.processor() or "unknown"


def _cores():
    """Cores this process may use: the affinity set, capped by OMP_NUM_THREADS when the host sets
    it (the GPU box gives one GPU's job 16 of its cores and exports OMP_NUM_THREADS=16)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return min(n, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else n


def oracle_rows():
    import oracle
    from guava_renderer_amd import camera, scenes
    cores = _cores()
    rows = []
    d = scenes.random_cloud(10000, 0)
    cam = camera.camera(256, 256)
    bg = np.zeros(32, np.float32)

    def proj_sort():
        st = oracle.preprocess(d["means3D"], d["scales"], d["rotations"], d["opacities"], None, cam["viewmatrix"],
                               cam["projmatrix"], 256, 256, cam["tanfovx"], cam["tanfovy"])
        oracle.bin_and_sort(st, 256, 256)

    def full(dd, W):
        c = camera.camera(W, W)
        return lambda: oracle.forward(dd["means3D"], dd["colors"], dd["opacities"], dd["scales"], dd["rotations"],
                                      None, c["viewmatrix"], c["projmatrix"], W, W, c["tanfovx"], c["tanfovy"], bg)

    for th in sorted({1, cores}):
        oracle.set_threads(th)
        t = _median_time(proj_sort, 3, 20)
        rows.append({"config": "C1 10k random, 256x256", "what": "preprocess + bin + stable sort", "threads": th,
                     "ms": round(1000 * t, 3)})
        t = _median_time(full(d, 256), 3, 20)
        rows.append({"config": "C1 10k random, 256x256", "what": "full forward render (32 ch)", "threads": th,
                     "ms": round(1000 * t, 3), "frames_per_s": round(1.0 / t, 2)})
    oracle.set_threads(cores)
    d2 = scenes.avatar_cloud(100000, seed=0)
    t = _median_time(full(d2, 512), 1, 5)
    rows.append({"config": "C2 100k avatar cloud, 512x512", "what": "full forward render (32 ch)", "threads": cores,
                 "ms": round(1000 * t, 2), "frames_per_s": round(1.0 / t, 3)})
    return rows


def reference_lbs_rows():
    ref_path = "/root/reference/models/modules/flame/lbs.py"
    if not os.path.exists(ref_path):
        return []
    import torch
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    spec = importlib.util.spec_from_file_location("ref_flame_lbs", ref_path)
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    torch.set_num_threads(8)
    V, J = 10595, 55
    rng = np.random.default_rng(0)
    parents = np.concatenate([[-1], rng.integers(0, np.arange(1, J))]).astype(np.int64)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))  # noqa: E731
    posedirs = t(rng.normal(0, 1e-3, ((J - 1) * 9, V * 3)))
    Jreg = rng.random((J, V)).astype(np.float32)
    Jreg /= Jreg.sum(1, keepdims=True)
    w = rng.random((V, J)).astype(np.float32) ** 8
    w /= w.sum(1, keepdims=True)
    rows = []
    for B in (1, 32):
        pose = t(rng.normal(0, 0.15, (B, J * 3)))
        v_shaped = t(rng.normal(0, 0.3, (B, V, 3)))
        fn = lambda: ref.lbs_wobeta(pose, v_shaped, posedirs, t(Jreg), torch.from_numpy(parents), t(w))  # noqa: E731
        with torch.no_grad():
            tm = _median_time(fn, 2, 10)
        rows.append({"config": f"reference lbs_wobeta V={V} J={J}", "what": f"torch CPU, batch {B}",
                     "threads": 8, "ms": round(1000 * tm, 2), "frames_per_s": round(B / tm, 1)})
    return rows


def main():
    out = {"host": platform.node(), "cpu": _cpu_model(), "affinity_cores": len(os.sched_getaffinity(0)),
           "os_cpu_count": os.cpu_count(), "cores_used": _cores(), "rows": oracle_rows() + reference_lbs_rows()}
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
