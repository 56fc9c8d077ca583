"""Instruction mix of the innermost loop (the one holding v_mfma) of a kernel in a hipcc -S file.
usage: loop_mix.py file.s mangled_kernel_name"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
i = s.index(sys.argv[2] + ":")
j = s.index(".Lfunc_end", i)
lines = s[i:j].splitlines()
blocks = []  # (label, header, [instrs])
cur = None
for l in lines:
    m = re.match(r"^(\.LBB\d+_\d+):(.*)", l)
    if m:
        hm = re.search(r"Header=BB(\d+_\d+) Depth=(\d+)", m.group(2))
        hdr = None
        if hm:
            hdr = "BB" + hm.group(1)
        if "Loop Header" in m.group(2):
            hdr = m.group(1).replace(".L", "")
        cur = [m.group(1), hdr, []]
        blocks.append(cur)
        continue
    t = l.strip()
    if cur is not None and t and not t.startswith(";") and not t.startswith("."):
        cur[2].append(t.split()[0])
mf = [b for b in blocks if any(x.startswith("v_mfma") for x in b[2])]
hdr = mf[0][1]
loop = [b for b in blocks if b[1] == hdr]
c = collections.Counter()
for b in loop:
    c.update(b[2])
print("loop header", hdr, "blocks", len(loop), "instrs", sum(c.values()))
cls = collections.Counter()
for k, v in c.items():
    key = "mfma" if k.startswith("v_mfma") else "valu" if k.startswith("v_") else "salu" if k.startswith("s_") and not k.startswith(("s_waitcnt", "s_cbranch", "s_branch", "s_nop", "s_load")) else "mem" if k.startswith(("global_", "buffer_", "ds_", "s_load")) else "ctl"
    cls[key] += v
print(dict(cls))
for k, v in c.most_common(40):
    print(f"{v:4d} {k}")
