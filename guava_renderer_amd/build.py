"""Builds guava_renderer_amd/lib/libgsr.so for gfx950 with hipcc (no torch headers involved).

    python -m guava_renderer_amd.build        # or via __graft_entry__.build()

-ffp-contract=off is part of the numerics contract: the kernels and the CPU oracle
evaluate the same expressions in the same order.
"""
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
OBJ_DIR = os.path.join(HERE, "lib", "obj")
LIB = os.path.join(LIB_DIR, "libgsr.so")
SOURCES = ["preprocess.hip", "binning.hip", "render_fwd.hip", "render_bwd.hip",
           "preprocess_bwd.hip", "deform.hip", "ehm.hip", "ssim.hip", "frames.hip", "capi.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("GSR_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}",
         "-Wno-unused-result", "-I" + CSRC, "-I" + os.path.join(os.path.dirname(HERE), "include")]


# per-source extras: no SLP packing in the render kernel (packed f32 VALU beside MFMAs costs more
# issue slots than the scalar pair, MI355X_MICROARCH.md "price of one filler")
EXTRA = {"render_fwd.hip": ["-fno-slp-vectorize"], "render_bwd.hip": ["-fno-slp-vectorize"]}


def source_hash():
    """SHA-256 (first 16 hex digits) over every HIP source, internal header and include/*.h, plus the
    compile flags: stamped into the library (gsr_version) so a stale prebuilt .so is detected at
    load time (_lib.load) instead of silently running old code."""
    h = hashlib.sha256()
    inc = os.path.join(os.path.dirname(HERE), "include")
    files = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".h")))
    files += sorted(os.path.join(inc, f) for f in os.listdir(inc) if f.endswith(".h"))
    for f in files:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    h.update(" ".join(f for f in FLAGS if not f.startswith("-I")).encode())  # (no paths: the tree moves)
    h.update(repr(sorted(EXTRA.items())).encode())
    return h.hexdigest()[:16]


def _newer(src_paths, dst):
    if not os.path.exists(dst):
        return True
    t = os.path.getmtime(dst)
    return any(os.path.getmtime(p) > t for p in src_paths)


def _compile(src):
    obj = os.path.join(OBJ_DIR, os.path.splitext(src)[0] + ".o")
    deps = [os.path.join(CSRC, src)] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    inc = os.path.join(os.path.dirname(HERE), "include")
    deps += [os.path.join(inc, h) for h in os.listdir(inc) if h.endswith(".h")]
    stamp = obj + ".hash"
    want = source_hash()
    stale = not os.path.exists(stamp) or open(stamp).read() != want
    if stale or _newer(deps, obj):
        cmd = [HIPCC] + FLAGS + EXTRA.get(src, []) + [f'-DGSR_SRC_HASH="{want}"', "-c", os.path.join(CSRC, src),
                                                      "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
        open(stamp, "w").write(want)
    return obj


def build(verbose=True, jobs=None):
    os.makedirs(OBJ_DIR, exist_ok=True)
    jobs = jobs or min(len(SOURCES), int(os.environ.get("MAX_JOBS", "8")))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(_compile, SOURCES))
    if _newer(objs, LIB):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[gsr] built {LIB}")
    return LIB


if __name__ == "__main__":
    build()
    sys.exit(0)
