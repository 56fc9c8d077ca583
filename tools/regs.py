"""Per-kernel register / spill / occupancy report of one HIP source (hipcc -Rpass-analysis):
    python tools/regs.py render_fwd.hip [-DFLAG ...]"""
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from guava_renderer_amd import build as b  # noqa: E402

src = sys.argv[1]
path = src if os.path.exists(src) else os.path.join(b.CSRC, src)
cmd = [b.HIPCC] + b.FLAGS + b.EXTRA.get(os.path.basename(src), []) + sys.argv[2:] + [
    '-DGSR_SRC_HASH="x"', "-c", path, "-o", "/tmp/_regs.o", "-Rpass-analysis=kernel-resource-usage"]
r = subprocess.run(cmd, capture_output=True, text=True)
cur = None
rows = []
for line in r.stderr.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    s = m.group(1).strip()
    if s.startswith("Function Name:"):
        name = s.split(":", 1)[1].strip()
        dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        cur = {"name": dm}
        rows.append(cur)
    elif cur is not None and ":" in s:
        k, v = s.split(":", 1)
        cur[k.strip()] = v.strip()
for c in rows:
    n = re.sub(r"\(gsr::Dims.*", "", c["name"]).replace("gsr::", "")
    print(f"{n[:90]:90s} V={c.get('VGPRs','?'):>4} A={c.get('AGPRs','?'):>3} Vspill={c.get('VGPRs Spill','?'):>4} "
          f"Sspill={c.get('SGPRs Spill','?'):>4} occ={c.get('Occupancy [waves/SIMD]','?')} lds={c.get('LDS Size [bytes/block]','?')}")
if r.returncode:
    print(r.stderr[-3000:])
