"""Effective shader clock per dispatch from one rocprofv3 run with
--pmc GRBM_GUI_ACTIVE --kernel-trace (MI355X_MICROARCH.md 'DVFS give-back':
GRBM_GUI_ACTIVE counts GPU-busy cycles summed over the 8 XCDs, so
clock = GRBM_GUI_ACTIVE / 8 / wall).  The profiler serialises dispatches
while it collects counters, so each kernel runs alone here.

    python3 tools/dispatch_clock.py gpurun_out/r02_c3_grbm --what "..." --out profiles/x.json
"""
import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--what", default="")
    ap.add_argument("--out", required=True)
    ap.add_argument("--kernels", default="fir_tile_kernel|loop_kernel|fll_sys_kernel")
    a = ap.parse_args()
    import re
    pat = re.compile(a.kernels)
    cnt = {}
    for fn in glob.glob(os.path.join(a.root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(fn, newline="")):
            if row.get("Counter_Name") == "GRBM_GUI_ACTIVE":
                k = row["Dispatch_Id"]
                cnt[k] = cnt.get(k, 0.0) + float(row["Counter_Value"])
    out = []
    for fn in glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(fn, newline="")):
            name = row.get("Kernel_Name", "")
            m = pat.search(name)
            if not m:
                continue
            k = row["Dispatch_Id"]
            ns = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
            g = cnt.get(k)
            out.append({"dispatch": int(k), "kernel": "qpsk::" + m.group(0), "ms": round(ns / 1e6, 3),
                        "GRBM_GUI_ACTIVE": g,
                        "eff_clock_GHz": round(g / 8 / ns, 3) if g else None})
    out.sort(key=lambda r: r["dispatch"])
    json.dump({"what": a.what, "dispatches": out}, open(a.out, "w"), indent=1)
    print(f"{len(out)} dispatches -> {a.out}")


if __name__ == "__main__":
    main()
