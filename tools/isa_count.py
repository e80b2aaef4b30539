#!/usr/bin/env python3
"""tools/isa_count.py -- instruction mix of a kernel's main loop in gfx950 ISA.

Usage: isa_count.py ISA.s KERNEL_SYMBOL [--per N] [--ops]

ISA.s: `hipcc --offload-arch=gfx950 --cuda-device-only -S` output built with
the Makefile's flags for that file (the FLL: -fno-slp-vectorize -mllvm
-misched=ilpmin).  The main loop is taken as the largest contiguous region
from a loop-header label to the first branch back to it (for fll_sys_kernel:
the do-while of four register-window blocks, fast path only; the exact redo
blocks sit after the back edge).  Counts are divided by --per (4 for the FLL:
four 8-sample blocks per iteration) and split into the categories DESIGN.md
3.3 uses: packed f32, f64 and conversions, DPP, hazard s_nop, other VALU,
scalar / branch, memory.
"""
import argparse
import collections
import re


def kernel_lines(path, name):
    lines = open(path).read().split('\n')
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ':'))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
    return lines[start:end]


def main_loop(lines):
    best = None
    for i, l in enumerate(lines):
        m = re.match(r'^(\.LBB\d+_\d+):.*Loop Header', l)
        if not m:
            continue
        lab = m.group(1)
        for j in range(i + 1, len(lines)):
            if re.search(r's_cbranch_\w+\s+' + re.escape(lab) + r'\b|s_branch\s+' + re.escape(lab) + r'\b',
                         lines[j]):
                if best is None or j - i > best[1] - best[0]:
                    best = (i, j, lab)
                break
    return best


def category(s):
    op = s.split()[0]
    if 'dpp' in s or 'row_' in s or 'quad_perm' in s:
        return 'dpp'
    if op.startswith('s_nop'):
        return 'hazard s_nop'
    if op.startswith('s_'):
        return 'scalar / branch'
    if op.startswith(('global_', 'ds_', 'buffer_', 'flat_')):
        return 'memory'
    if 'f64' in op or 'cvt' in op:
        return 'f64 / conversion'
    if op.startswith('v_pk_'):
        return 'packed f32'
    return 'other VALU'


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('isa')
    ap.add_argument('kernel')
    ap.add_argument('--per', type=float, default=1.0)
    ap.add_argument('--ops', action='store_true')
    a = ap.parse_args()
    lines = kernel_lines(a.isa, a.kernel)
    i, j, lab = main_loop(lines)
    cat, ops, n = collections.Counter(), collections.Counter(), 0
    for l in lines[i:j + 1]:
        s = l.strip()
        if not s or s.startswith(';') or s.startswith('.') or s.endswith(':'):
            continue
        n += 1
        cat[category(s)] += 1
        ops[s.split()[0]] += 1
    print(f'{a.kernel}: loop {lab}, ISA lines {i}-{j} of the kernel, {n} instructions, '
          f'{n / a.per:.1f} per unit (/{a.per:g})')
    for k, v in cat.most_common():
        print(f'  {k:18s} {v / a.per:7.2f}')
    if a.ops:
        for k, v in ops.most_common():
            print(f'    {k:26s} {v / a.per:7.2f}')


if __name__ == '__main__':
    main()
