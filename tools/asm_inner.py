"""The smallest loop (backward branch) of a kernel that contains an MFMA, with its instruction mix
and the sequence:  python tools/asm_inner.py file.s <mangled-name-prefix> [--list]"""
import collections
import re
import sys

s = open(sys.argv[1]).read().split('\n')
key = sys.argv[2]
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
best = None
for i, l in enumerate(body):
    m = re.match(r'^\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)', l)
    if m and m.group(2) in labels and labels[m.group(2)] < i:
        seg = [x.strip() for x in body[labels[m.group(2)]:i + 1]
               if (x.startswith('\t') and not x.strip().startswith(('.', ';'))) or x.startswith('.LBB')]
        if any('mfma' in x for x in seg) and (best is None or len(seg) < len(best)):
            best = seg
ins = [x for x in best if not x.startswith('.LBB')]
c = collections.Counter(x.split()[0] for x in ins)
valu = sum(v for k, v in c.items() if k.startswith('v_') and 'mfma' not in k)
salu = sum(v for k, v in c.items() if k.startswith('s_') and not k.startswith(('s_waitcnt', 's_nop')))
mfma = sum(v for k, v in c.items() if 'mfma' in k)
print(f'{len(ins)} instructions, VALU {valu}, SALU(+branch) {salu}, MFMA {mfma}, waitcnt {c["s_waitcnt"]}, '
      f'VMEM {sum(v for k, v in c.items() if k.startswith(("buffer_", "global_")))}, '
      f'LDS {sum(v for k, v in c.items() if k.startswith("ds_"))}')
for k, v in c.most_common(70):
    print(f'   {k:32s} {v}')
if '--list' in sys.argv:
    print('\n'.join(best))
