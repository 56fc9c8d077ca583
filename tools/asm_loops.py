"""Innermost-loop instruction counts of one kernel in a hipcc -S file: every backward branch
(label defined earlier in the kernel) is a loop; prints its size and instruction histogram.
    python tools/asm_loops.py file.s <mangled-name-substring> [top]"""
import collections
import re
import sys

s = open(sys.argv[1]).read().split('\n')
key = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
start = next(i for i, l in enumerate(s) if l.startswith(key) and ':' in l)
body = []
for l in s[start + 1:]:
    if l.startswith('.Lfunc_end'):
        break
    body.append(l)
labels = {}
for i, l in enumerate(body):
    m = re.match(r'^(\.LBB\w+):', l)
    if m:
        labels[m.group(1)] = i
loops = []
for i, l in enumerate(body):
    m = re.match(r'^\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)', l)
    if m and m.group(2) in labels and labels[m.group(2)] < i:
        seg = [x.strip() for x in body[labels[m.group(2)]:i + 1] if x.startswith('\t') and not x.strip().startswith(('.', ';'))]
        loops.append((len(seg), m.group(2), seg))
for n, lab, seg in sorted(loops, reverse=True)[:3]:
    c = collections.Counter(x.split()[0] for x in seg)
    valu = sum(v for k, v in c.items() if k.startswith('v_') and 'mfma' not in k)
    salu = sum(v for k, v in c.items() if k.startswith('s_') and not k.startswith(('s_waitcnt', 's_nop', 's_cbranch', 's_branch')))
    print(f'loop {lab}: {n} instructions, VALU {valu}, SALU {salu}, MFMA {sum(v for k, v in c.items() if "mfma" in k)}')
    for k, v in c.most_common(top):
        print(f'   {k:32s} {v}')
