"""Build an A/B variant of libgsr.so into guava_renderer_amd/lib/ab/libgsr_<tag>.so:
    python tools/build_ab.py <tag> [src.hip=path/to/replacement.hip ...] [-DFLAG ...]
Every source is compiled with the tree's flags plus -DGSR_TUNING (the tuning switches and timing
ablations read from the environment: gsr_internal.h tune_env) and the given -D flags; a replaced
source comes from the given path.  The product library (guava_renderer_amd/build.py) never sets
GSR_TUNING."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from guava_renderer_amd import build as b  # noqa: E402

tag = sys.argv[1]
repl = dict(a.split("=", 1) for a in sys.argv[2:] if "=" in a and not a.startswith("-D"))
defs = ["-DGSR_TUNING"] + [a for a in sys.argv[2:] if a.startswith("-D")]
out_dir = os.path.join(os.path.dirname(b.LIB), "ab")
os.makedirs(out_dir, exist_ok=True)
want = b.source_hash()
objs = []
for src in b.SOURCES:
    obj = os.path.join(b.OBJ_DIR, os.path.splitext(src)[0] + ".o")
    if src in repl or defs:
        path = repl.get(src, os.path.join(b.CSRC, src))
        obj = os.path.join(out_dir, f"{tag}_{os.path.splitext(src)[0]}.o")
        cmd = [b.HIPCC] + b.FLAGS + b.EXTRA.get(src, []) + defs + [f'-DGSR_SRC_HASH="{want}"', "-I", b.CSRC, "-c",
                                                                     path, "-o", obj]
        subprocess.run(cmd, check=True, capture_output=True)
    objs.append(obj)
lib = os.path.join(out_dir, f"libgsr_{tag}.so")
subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", lib] + objs, check=True)
print(lib)
