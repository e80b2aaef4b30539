#!/usr/bin/env python3
"""tools/sq_breakdown.py -- per-kernel SQ wave-cycle breakdown from a rocprofv3
--pmc run (the SQLite results.db rocprofv3 7.x writes by default, or a
counter_collection.csv): each counter summed over the kernel's dispatches and
shown as a fraction of SQ_WAVE_CYCLES (WAIT_ANY + WAIT_INST_ANY +
ACTIVE_INST_ANY ~= WAVE_CYCLES, all in quad-cycles; MI355X_MICROARCH.md,
rocprofv3 PMC slots).

Usage: sq_breakdown.py RESULTS.db|CSV [KERNEL_SUBSTRING ...]"""
import collections
import csv
import sqlite3
import sys


def rows(path):
    if path.endswith(".db"):
        db = sqlite3.connect(path)
        for k, d, c, v in db.execute("select kernel_name, dispatch_id, counter_name, value from counters_collection"):
            yield k, d, c, float(v)
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                yield r.get("Kernel_Name", ""), r.get("Dispatch_Id"), r["Counter_Name"], float(r["Counter_Value"])


def main():
    path, keys = sys.argv[1], sys.argv[2:]
    tot = collections.defaultdict(collections.Counter)
    disp = collections.defaultdict(set)
    for k, d, c, v in rows(path):
        name = next((s for s in keys if s in k), None) if keys else k[:60]
        if name is None:
            continue
        tot[name][c] += v
        disp[name].add(d)
    for name, c in tot.items():
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        print(f"== {name}: {len(disp[name])} dispatches")
        for cn, v in sorted(c.items()):
            frac = f"{v / wc:7.3f} of WAVE_CYCLES" if wc and cn.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
            print(f"  {cn:24s} {v:18.0f}  {frac}")
        if c.get("SQ_INSTS_VALU") and wc:
            print(f"  wave-cycles per VALU instruction: {4 * wc / c['SQ_INSTS_VALU']:.2f}")


if __name__ == "__main__":
    main()
