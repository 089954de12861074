#!/usr/bin/env python3
"""Per kernel in a gfx950 .s file: the number of global/buffer loads issued before each
`s_waitcnt vmcnt` (a 1 repeated in a loop = one exposed memory latency per iteration)."""
import re
import sys

s = open(sys.argv[1]).read()
for m in re.finditer(r'^(_Z\S+):[^\n]*\n(.*?)\n\s*s_endpgm', s, re.S | re.M):
    name = re.sub(r'^_ZN2vx12_GLOBAL__N_1\d+', '', m.group(1))[:40]
    seq, cur, loops = [], 0, 0
    for ln in m.group(2).split('\n'):
        if re.search(r'\b(global|buffer)_load', ln):
            cur += 1
        elif 's_waitcnt' in ln and 'vmcnt' in ln:
            seq.append(cur)
            cur = 0
        elif re.match(r'\s*s_cbranch', ln):
            seq.append('|')
    print(f"{name:40s} {' '.join(map(str, seq))[:300]}")
