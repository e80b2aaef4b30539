"""bench.py's stdout line stays within what the driver parses.

Round 4's single line grew to 26.3 KB (per-launch statistics, clock ranges,
FIR phase samples, three full sub-records) and the driver left it unparsed;
round 3's 19.8 KB line parsed.  The line now carries only the driver's keys,
the roofline, cpu_baseline, parity counts and BER (GPU and CPU) per record;
the full record goes to the detail file.  These tests build the line from a
canned full run (profiles/r04d_bench_default.json: the 26.3 KB record itself)
and from a synthetic worst case.
"""
import copy
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.argv = sys.argv[:1]
import bench  # noqa: E402

CANNED = os.path.join(ROOT, "profiles", "r04d_bench_default.json")
DRIVER_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
               "scaling", "vs_baseline", "dtype", "data", "config")


def canned():
    with open(CANNED) as f:
        rec = json.load(f)
    ber = {"bit_errors": 1, "bits": 2, "ber": 0.5, "lost_windows": 0, "symbol_slips": 0, "equal": True}
    rec["ber_cpu"] = ber
    for r in rec["sub_records"].values():
        r["ber_cpu"] = dict(ber)
    rec["sub_records"]["c3_glibc"] = copy.deepcopy(rec["sub_records"]["c4"])
    return rec


def test_canned_full_run_line_is_bounded_and_complete():
    full = canned()
    assert len(json.dumps(full)) > 20_000          # the record that did not parse
    s = bench.dump_line(bench.compact_record(full, "bench_detail.json"))
    assert "\n" not in s
    assert len(s) <= 12_000
    line = json.loads(s)
    for k in DRIVER_KEYS:
        assert k in line, k
    assert line["value"] == full["value"]
    roof = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in roof, k
    cpu = line["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cpu, k
    par = line["parity"]
    assert par["libm_oracle"]["mismatching"] == 0 and par["libm_oracle"]["streams"] > 0
    assert line["ber"]["bits"] > 0 and line["ber_cpu"]["equal"] is True
    assert line["detail"] == "bench_detail.json"
    assert set(line["sub_records"]) == {"c2", "c4", "c5", "c3_glibc"}
    for key, r in line["sub_records"].items():
        for k in ("value", "ms_per_step", "roofline", "cpu_baseline", "parity", "ber", "ber_cpu"):
            assert k in r, (key, k)
    # nothing of the per-launch detail reaches the line
    for k in ("launch_stats", "phases", "clock_ghz_range", "framer", "host_ring", "mismatch_examples"):
        assert f'"{k}"' not in s, k


DROP_IN = {
    "s1_host": {"kind": "drop_in", "value": 61.2, "unit": "MSa/s", "ms_per_step": 17.1, "steps": 10, "warmup": 2,
                "config": {"workload": "1 stream x 2^20 samples, sps 8, 65 taps, host memory, "
                                       "qpsk_demod_process(MEM_HOST) with S = 1 (the INTEGRATION.md shim)"},
                "cpu_single_core": 59.5, "parity": {"libm_oracle": {"streams": 1, "mismatching": 0}},
                "note": "x" * 300},
    "host_ring_c3": {"kind": "drop_in", "value": 6500.0, "unit": "MSa/s", "ms_per_step": 660.0, "steps": 2,
                     "warmup": 1, "h2d_GBps": 52.0,
                     "config": {"workload": "C3 from host memory: 4096 streams x 2^20 samples per step through "
                                            "the pinned ring (qpsk_rx_*), 4 chunks of 262144 samples per "
                                            "stream, depth 4"},
                     "parity": {"libm_oracle": {"streams": 2, "mismatching": 0}}, "note": "y" * 300},
}


def test_full_line_with_drop_in_records_stays_bounded_untrimmed():
    """The round-6 line: the four config sub-records plus the two drop-in
    shapes (s1_host, host_ring_c3) fit the 12 KB bound with nothing trimmed:
    every sub-record keeps its kernel table, and the drop-in records keep
    value, cpu_single_core and parity."""
    full = canned()
    full["sub_records"].update(copy.deepcopy(DROP_IN))
    line = bench.compact_record(full, "bench_detail.json")
    untrimmed = json.dumps(line, separators=(",", ":"))
    s = bench.dump_line(line)
    assert s == untrimmed and len(s) <= bench.LINE_MAX_BYTES, len(untrimmed)
    got = json.loads(s)["sub_records"]
    assert got["s1_host"]["cpu_single_core"] == 59.5 and got["s1_host"]["value"] == 61.2
    assert got["s1_host"]["parity"]["libm_oracle"]["mismatching"] == 0
    assert got["host_ring_c3"]["h2d_GBps"] == 52.0
    assert "note" not in got["s1_host"] and "kernels" in got["c2"]
    # a leg that failed keeps its error text in the line
    full["sub_records"]["s1_host"] = {"kind": "drop_in", "error": "RuntimeError: boom"}
    got = json.loads(bench.dump_line(bench.compact_record(full, "d.json")))["sub_records"]
    assert got["s1_host"]["error"] == "RuntimeError: boom"


def test_oversized_sub_records_are_trimmed_not_fatal():
    full = canned()
    for i in range(40):
        full["sub_records"][f"x{i}"] = copy.deepcopy(full["sub_records"]["c5"])
    s = bench.dump_line(bench.compact_record(full, "d.json"))
    line = json.loads(s)
    assert len(s) <= bench.LINE_MAX_BYTES
    assert line["value"] == full["value"] and "roofline" in line and "cpu_baseline" in line
    assert all("value" in r for r in line["sub_records"].values())


def test_oversized_headline_falls_back_to_driver_keys(capsys):
    """A headline too big by itself (nothing left to trim in sub-records) is
    cut down to the driver's keys + roofline + cpu_baseline, with a warning on
    stderr, instead of leaving the driver an unparsable line."""
    full = canned()
    full.pop("sub_records")
    full["config"] = dict(full["config"], padding="x" * 20_000)   # the driver's own keys overflow
    s = bench.dump_line(bench.compact_record(full, "d.json"))
    line = json.loads(s)
    assert line["truncated"] is True and line["detail"] == "d.json"
    assert line["value"] == full["value"] and "metric" in line
    assert "bench.py: stdout line" in capsys.readouterr().err
    full["config"] = dict(full["config"], padding="x")
    full["stages_ms"] = {f"k{i}": i for i in range(2000)}            # a bloated body only
    line = json.loads(bench.dump_line(bench.compact_record(full, "d.json")))
    assert len(json.dumps(line, separators=(",", ":"))) <= bench.LINE_MAX_BYTES
    assert "roofline" in line and "cpu_baseline" in line and line["truncated"] is True


def test_missing_legs_serialise():
    """--timed-only: no parity, no cpu baseline, no sub-records."""
    full = canned()
    for k in ("cpu_baseline", "parity_vs_libm_oracle", "sub_records", "ber_cpu"):
        full.pop(k)
    full["parity_vs_portable_oracle"] = full["parity_steady_state"] = "not checked"
    line = json.loads(bench.dump_line(bench.compact_record(full, "d.json")))
    assert line["cpu_baseline"] is None and line["parity"] == "not checked"
    assert "sub_records" not in line


@pytest.mark.parametrize("n", [0, 1, 40])
def test_ber_counter_accepts_host_rows(n):
    """ber_after_lock counts the CPU oracle's numpy rows like device rows."""
    import numpy as np
    rng = np.random.default_rng(5)
    tx = rng.integers(0, 2, 30000).astype(np.uint8)
    rx = tx[2:].copy()
    if n:
        rx[rng.choice(np.arange(9000, 29000), n, replace=False)] ^= 1
    bits = np.packbits(rx)[None, :]
    e, tot, lost, slips = bench.ber_after_lock(bits, np.array([rx.size]), np.packbits(tx)[None, :], 1)
    assert slips == 0 and tot > 15000
    assert e + 64 * lost >= min(n, 1) and e <= n
