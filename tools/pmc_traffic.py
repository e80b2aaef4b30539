"""HBM bytes per launch of one kernel from two rocprofv3 PMC passes.

Usage (on the GPU box, one pass per counter, as MI355X_MICROARCH.md's HBM
section prescribes -- FETCH_SIZE and WRITE_SIZE do not fit one TCC pass):

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -- python3 bench.py ...
    python3 tools/pmc_traffic.py --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write \
        --kernel fir_tile_kernel --algo-bytes B --out profiles/pmc_fir_c2.json

Corrections (MI355X_MICROARCH.md "HBM"): FETCH_SIZE/WRITE_SIZE are reported in
KiB; on gfx950 FETCH_SIZE counts exactly half the bytes of a wide (16 B/lane)
streaming read, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics


def per_dispatch(root: str, counter: str, kernel_re: str):
    files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {root}")
    vals = {}
    pat = re.compile(kernel_re)
    for fn in files:
        with open(fn, newline="") as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                if not pat.search(row.get("Kernel_Name", "")):
                    continue
                key = (fn, row.get("Dispatch_Id"))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for kernel /{kernel_re}/ under {root}")
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", required=True, help="regex on Kernel_Name")
    ap.add_argument("--algo-bytes", type=float, required=True,
                    help="algorithmic bytes per launch (DESIGN.md)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    write = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    # drop the warmup/parity dispatches of other sizes: keep the modal size
    f_med = statistics.median(fetch)
    w_med = statistics.median(write)
    rd = 2.0 * f_med * 1024.0
    wr = w_med * 1024.0
    out = {
        "kernel": a.kernel,
        "dispatches": {"fetch": len(fetch), "write": len(write)},
        "FETCH_SIZE_KiB_median": f_med,
        "WRITE_SIZE_KiB_median": w_med,
        "correction": "read bytes = 2 x FETCH_SIZE x 1024 (gfx950 wide-read half count); "
                      "write bytes = WRITE_SIZE x 1024",
        "hbm_read_bytes_per_launch": rd,
        "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr,
        "algorithmic_bytes_per_launch": a.algo_bytes,
        "traffic_over_algorithmic": (rd + wr) / a.algo_bytes,
    }
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
