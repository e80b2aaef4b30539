#!/usr/bin/env python3
"""tools/issue_model.py -- in-order issue model of one wave's loops in gfx950 ISA.

Usage: issue_model.py ISA.s KERNEL_SYMBOL [--trace LABEL] [--cadence 5.1]
                      [--latency 8.3] [--lds 60]

ISA.s: `hipcc --offload-arch=gfx950 --cuda-device-only -S` output (the same
flags as the Makefile, including -amdgpu-sched-strategy for the loop kernel).
Lists every innermost loop of the kernel with its VALU / LDS instruction
counts and the modelled cycles per iteration; --trace prints one loop's
schedule instruction by instruction.

The model (constants from tools/isa_bench.hip on MI355X):
a wave issues in order; a VALU instruction issues `cadence` cycles after the
previous one at the earliest, and `latency` cycles after the instruction
that produces one of its operands; an LDS read's result is ready `lds` cycles
after it issues; s_waitcnt waits for every outstanding LDS read; scalar
instructions are free.  It reproduces the stamped loop probe's uniform-loop
cycles per symbol within ~5 % for the M&M and Costas waves.
"""
import argparse
import re


def regs(tok):
    out = []
    for m in re.finditer(r'([vs])\[(\d+):(\d+)\]|([vs])(\d+)\b|\b(vcc)\b', tok):
        if m.group(1):
            out += [f'{m.group(1)}{i}' for i in range(int(m.group(2)), int(m.group(3)) + 1)]
        elif m.group(4):
            out.append(f'{m.group(4)}{m.group(5)}')
        else:
            out.append('vcc')
    return out


def simulate(body, cadence, latency, lds, iters=4, trace=False):
    ready, outstanding = {}, []
    t, last, starts = 0.0, -1e9, []
    for it in range(iters):
        starts.append(t)
        for ins in body:
            op = ins.split()[0]
            ops = [o.strip() for o in ins[len(op):].split(',')]
            if op.startswith('s_waitcnt'):
                if outstanding:
                    t = max(t, max(outstanding))
                    outstanding = []
                continue
            if op.startswith('s_'):
                continue
            if op.startswith('v_cmp') and '_e32' in op:
                dst, srcs = ['vcc'], ops
            elif op.startswith('ds_write'):
                dst, srcs = [], ops
            else:
                dst, srcs = regs(ops[0]), ops[1:]
            if 'fmac' in op:
                srcs = srcs + [ops[0]]
            if 'cndmask' in op and '_e32' in op:
                srcs = srcs + ['vcc']
            need = max([ready.get(r, 0.0) for s in srcs for r in regs(s)] + [0.0])
            issue = max(last + cadence, need, t)
            last = t = issue
            lat = lds if op.startswith('ds_read') else latency
            for r in dst:
                ready[r] = issue + lat
            if op.startswith('ds_read'):
                outstanding.append(issue + lds)
            if trace and it == iters - 2:
                print(f'{issue - starts[-1]:8.1f}  {ins}')
    return [starts[i + 1] - starts[i] for i in range(len(starts) - 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('isa')
    ap.add_argument('kernel')
    ap.add_argument('--trace')
    ap.add_argument('--cadence', type=float, default=5.1)
    ap.add_argument('--latency', type=float, default=8.3)
    ap.add_argument('--lds', type=float, default=60.0)
    a = ap.parse_args()
    L = open(a.isa).read().splitlines()
    st = next(i for i, l in enumerate(L) if l.startswith(a.kernel + ':'))
    en = next(i for i in range(st + 1, len(L)) if L[i].startswith('.Lfunc_end'))
    for i in range(st, en):
        m = re.match(r'^(\.LBB\d+_\d+):', L[i])
        if not m or not ('Inner Loop Header' in L[i] or 'Inner Loop Header' in L[i + 1]):
            continue
        lab = m.group(1)
        j = next((k for k in range(i + 1, en)
                  if re.search(r's_(cbranch_\w+|branch) ' + re.escape(lab) + r'$', L[k])), None)
        if j is None:
            continue
        body = [l.strip() for l in L[i + 1:j + 1]
                if l.strip() and not l.strip().startswith((';', '.', 's_cbranch', 's_branch'))]
        nv = sum(b.startswith('v_') for b in body)
        nd = sum(b.startswith('ds_') for b in body)
        cyc = simulate(body, a.cadence, a.latency, a.lds, trace=(a.trace == lab))
        print(f'{lab}: ISA lines {i + 1}-{j + 1}, {nv} VALU, {nd} LDS, modelled {cyc[-1]:.1f} cycles per iteration')


if __name__ == '__main__':
    main()
