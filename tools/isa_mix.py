"""Instruction mix of kernels in a hipcc --save-temps .s file (dev aid).
usage: python tools/isa_mix.py file.s <kernel-name-substring>"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
for m in re.finditer(r'^(\S*' + pat + r'\S*):.*$', s, re.M):
    n = m.group(1)
    end = s.index('.Lfunc_end', m.end())
    c = collections.Counter()
    for line in s[m.end():end].split('\n'):
        line = line.strip()
        if not line or line[0] in ';.' or line.endswith(':'):
            continue
        c[line.split()[0]] += 1
    print(n, 'total', sum(c.values()), 'valu', sum(x for k, x in c.items() if k.startswith('v_')))
    print(' ', c.most_common(30))
    for key in ['num_vgpr', 'num_agpr', 'private_seg_size']:
        mm = re.search(re.escape(n) + r'\.' + key + r', (\d+)', s)
        if mm:
            print('  ', key, mm.group(1))
