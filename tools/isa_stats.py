#!/usr/bin/env python3
"""Static ISA statistics of one kernel in a hipcc -S listing (gfx950).

Prints, for the kernel whose mangled name contains PATTERN, the counts of
spill-related instructions (v_readlane / v_writelane: SGPR spills to VGPR
lanes, both VALU; scratch_*: VGPR spills) and of the pair arithmetic, overall
and per loop (a label that a later s_cbranch jumps back to), so a spill that
sits inside a hot loop shows up as VALU work per iteration.

usage: hipcc --offload-arch=gfx950 -O3 -S --cuda-device-only x.hip -o x.s
       isa_stats.py x.s PATTERN [--loops]
"""
import collections
import re
import sys


def function_body(lines, pat):
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r'^(_Z\S*%s\S*):' % re.escape(pat), l):
            start = i
        elif start is not None and l.startswith('.Lfunc_end'):
            return lines[start:i]
    raise SystemExit('kernel %r not found' % pat)


KEYS = [('readlane', r'\bv_readlane_b32'), ('writelane', r'\bv_writelane_b32'),
        ('scratch_ld', r'\bscratch_load'), ('scratch_st', r'\bscratch_store'),
        ('v_exp_f32', r'\bv_exp_f32'), ('v_pk_fma_f32', r'\bv_pk_fma_f32'),
        ('valu', r'^\s+v_'), ('salu', r'^\s+s_(?!load|waitcnt|cbranch|branch|nop|barrier)'),
        ('s_load', r'^\s+s_load'), ('vmem', r'^\s+(global|buffer|flat)_')]


def count(block):
    c = collections.Counter()
    for l in block:
        for k, p in KEYS:
            if re.search(p, l):
                c[k] += 1
    return c


def main():
    path, pat = sys.argv[1], sys.argv[2]
    body = function_body(open(path).read().splitlines(), pat)
    print(body[0].split(':')[0], 'lines', len(body))
    print('  total', dict(count(body)))
    if '--loops' not in sys.argv:
        return
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r'^(\.LBB\S+):', l)
        if m:
            labels[m.group(1)] = i
    for i, l in enumerate(body):
        m = re.search(r's_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)', l)
        if not m:
            continue
        tgt = m.group(1) or m.group(2)
        j = labels.get(tgt)
        if j is not None and j < i:
            c = count(body[j:i + 1])
            print('  loop %s lines %d-%d (%d): %s' % (tgt, j, i, i - j, dict(c)))


if __name__ == '__main__':
    main()
