#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in a hipcc -S listing
(VALU / SALU / LDS / global / DPP / v_cndmask), with the block's source-line hints."""
import re
import sys


def main(path, pat):
    lines = open(path).read().split('\n')
    start = next(i for i, l in enumerate(lines) if re.match(r'^\S*' + pat + r'\S*:', l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
    blocks, cur = [], None
    for l in lines[start:end]:
        t = l.strip()
        if re.match(r'^[.\w$]+:', t):
            cur = {'name': t.split(':')[0], 'v': 0, 's': 0, 'ds': 0, 'gl': 0, 'dpp': 0, 'cnd': 0, 'loc': set()}
            blocks.append(cur)
            continue
        if cur is None or not t or t.startswith('.') or t.startswith(';'):
            m = re.search(r'qpb_gi.hip:(\d+)', t)
            if m and cur is not None:
                cur['loc'].add(int(m.group(1)))
            continue
        op = t.split()[0]
        if op.startswith('v_'):
            cur['v'] += 1
            cur['dpp'] += 'dpp' in t or 'row_' in t
            cur['cnd'] += op.startswith('v_cndmask')
        elif op.startswith('s_'):
            cur['s'] += 1
        elif op.startswith('ds_'):
            cur['ds'] += 1
        elif op.startswith(('global_', 'buffer_')):
            cur['gl'] += 1
    tot = dict(v=0, s=0, ds=0, gl=0, dpp=0, cnd=0)
    for b in blocks:
        loc = sorted(b['loc'])
        print(f"{b['name']:14s} v={b['v']:5d} s={b['s']:4d} ds={b['ds']:4d} gl={b['gl']:3d} dpp={b['dpp']:4d} "
              f"cnd={b['cnd']:4d} lines {loc[0] if loc else '-'}..{loc[-1] if loc else '-'}")
        for k in tot:
            tot[k] += b[k]
    print('total', tot)


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
