#!/bin/bash
# Register / scratch usage per kernel of one HIP source: tools/kres.sh file.hip [extra hipcc flags]
f=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I guava_renderer_amd/csrc -I include "$@" -c "$f" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); print(); print(cur[:70], end=" ")
        continue
    for key in ("VGPRs:", "VGPRs Spill:", "ScratchSize [bytes/lane]:", "Occupancy [waves/SIMD]:"):
        m = re.search(re.escape(key) + r" (\d+)", line)
        if m: print(key.split()[0] + "=" + m.group(1), end=" ")
    if "error" in line: print(line.strip())
print()'
