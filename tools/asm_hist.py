"""Instruction histogram of one kernel in a hipcc -S device assembly file:
python tools/asm_hist.py file.s <mangled-name-substring> [top]"""
import collections
import sys

s = open(sys.argv[1]).read().split('\n')
key = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
start = next(i for i, l in enumerate(s) if l.startswith(key) or (key in l and l.endswith(':') and not l.startswith('\t')))
body = []
for l in s[start + 1:]:
    if l.startswith('.Lfunc_end'):
        break
    body.append(l)
ins = [l.strip() for l in body if l.startswith('\t') and not l.strip().startswith(('.', ';'))]
print(s[start], 'instructions:', len(ins))
c = collections.Counter(x.split()[0] for x in ins)
for k, v in c.most_common(top):
    print(f'{k:32s} {v}')
