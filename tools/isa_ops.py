#!/usr/bin/env python3
"""Instruction histogram of one kernel in a hipcc -S listing.
Usage: tools/isa_ops.py file.s mangled-substring [topN]"""
import collections
import sys

s = open(sys.argv[1]).read()
key = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
name_line = [ln for ln in s.splitlines() if key in ln and ln.split(';')[0].rstrip().endswith(':')
             and not ln.startswith('.')][0]
i = s.index('\n' + name_line) + 1
j = s.index('.Lfunc_end', i)
ops = collections.Counter()
for line in s[i:j].splitlines():
    t = line.strip().split()
    if not t or t[0].startswith(('.', ';')) or t[0].endswith(':'):
        continue
    ops[t[0]] += 1
cls = collections.Counter()
for k, v in ops.items():
    c = 'valu_f64' if k.startswith('v_') and 'f64' in k else 'valu' if k.startswith('v_') else \
        'salu' if k.startswith('s_') else 'lds' if k.startswith('ds_') else 'vmem' if k.startswith(('global_', 'buffer_', 'scratch_')) else 'other'
    cls[c] += v
print(name_line, 'total', sum(ops.values()), dict(cls))
for k, v in ops.most_common(top):
    print(f'{k:28s}{v}')
