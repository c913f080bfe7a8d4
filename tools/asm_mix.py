#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc -S listing, split into
setup (before the outermost loop), loop (blocks tagged 'in Loop' / the loop
header, depth >= 1) and tail.  usage: asm_mix.py file.s kernel-name-regex"""
import collections
import re
import sys


def main(path, pat):
    L = open(path).read().split('\n')
    s = next(i for i, l in enumerate(L) if re.match(r'^' + pat + r'\S*:', l))
    e = next(i for i in range(s, len(L)) if L[i].startswith('.Lfunc_end'))
    region, seen_loop = 'setup', False
    mix = {k: collections.Counter() for k in ('setup', 'loop', 'tail')}
    for l in L[s:e]:
        t = l.strip()
        if re.match(r'^[.\w$]+:', t):
            if 'Loop' in t:
                region, seen_loop = 'loop', True
            else:
                region = 'tail' if seen_loop else 'setup'
            continue
        if not t or t[0] in '.;':
            continue
        op = t.split()[0]
        c = mix[region]
        if op.startswith('v_'):
            c['VALU'] += 1
            if 'dpp' in t or 'row_' in t or 'quad_perm' in t:
                c['dpp'] += 1
            if op.startswith('v_cndmask'):
                c['cndmask'] += 1
            if '_f64' in op:
                c['f64'] += 1
        elif op.startswith('s_'):
            c['SALU/branch'] += 1
        elif op.startswith('ds_'):
            c['LDS'] += 1
        elif op.startswith(('global_', 'buffer_', 'scratch_')):
            c['VMEM'] += 1
    for k, c in mix.items():
        print(f"{k:6s}", dict(c))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
