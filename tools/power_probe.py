"""tools/power_probe.py -- socket power, energy and GFX clock while the demod
runs serial calls (FIR then loop, back to back) and pipelined calls (FIR of
call k+1 beside the loop of call k).  Diagnostic for DESIGN.md 6 ("What bounds
C3"): is the pipelined step limited by the chip's power budget?

Usage: power_probe.py [config] [calls]   (config: c3 (default), c2, c5)
Writes gpurun_out/power_<config>.csv (t_s, phase, watts, gfx_mhz) and prints
one summary line per phase.  Reads the SMU through amdsmi (read-only).
"""
import os
import sys
import threading
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "qpsk-modulator-demodulator_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))
import qpsk_amd as Q  # noqa: E402
from bench import ALPHA, CONFIGS, FS  # noqa: E402

import amdsmi  # noqa: E402

key = sys.argv[1] if len(sys.argv) > 1 else "c3"
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 8
cfg = CONFIGS[key]
S, n, sps, span = cfg["streams"], 1 << 20, cfg["sps"], cfg["span"]
rs = FS // sps

amdsmi.amdsmi_init()
handles = amdsmi.amdsmi_get_processor_handles()


def read(h):
    pw = amdsmi.amdsmi_get_power_info(h)
    w = pw.get("current_socket_power")
    if not isinstance(w, (int, float)):
        w = pw.get("average_socket_power")
    ck = amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX)
    return float(w), float(ck.get("clk", 0))


def energy(h):
    e = amdsmi.amdsmi_get_energy_count(h)
    acc = e.get("energy_accumulator", e.get("power"))
    return float(acc) * float(e.get("counter_resolution", 1.0)) * 1e-6   # uJ -> J


print("power info keys:", sorted(amdsmi.amdsmi_get_power_info(handles[0]).keys()), flush=True)
# the card this process uses is the one whose power rises under load; sample all
samples = []          # (t, phase, [(w, mhz) per handle])
phase = ["idle"]
stop = threading.Event()


def sampler():
    while not stop.is_set():
        t = time.perf_counter()
        row = []
        for h in handles:
            try:
                row.append(read(h))
            except Exception:   # noqa: BLE001 -- a card we may not read
                row.append((float("nan"), float("nan")))
        samples.append((t, phase[0], row))
        time.sleep(0.001)


iq, _ = Q.synth_generate(S, n, FS, rs, rrc_alpha=ALPHA, rrc_span=span, seed=0x5159534B, lo_ppm=1.0,
                         cfo_hz=5000.0 if cfg["impaired"] else 0.0, multipath=cfg["impaired"],
                         esn0_db=20.0 if cfg["impaired"] else None, device=0)
p = Q.params(FS, rs, ALPHA, span, enable_fll=cfg["fll"], device=0, max_samples_per_call=n)
d = Q.BatchDemodulator(S, p)
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
d.set_stream(stream.cuda_stream)
ms = d.max_symbols(n)
bits = torch.zeros((S, (2 * ms + 7) // 8 + 64), dtype=torch.uint8, device="cuda")
nbits = torch.zeros(S, dtype=torch.int64, device="cuda")
d.enable_timing(True)
for _ in range(2):
    d.process_device(iq, n, bits, nbits)
torch.cuda.synchronize()

th = threading.Thread(target=sampler, daemon=True)
th.start()
time.sleep(0.3)
results = {}
for name in ("serial", "pipelined", "serial2"):
    e0 = [energy(h) for h in handles]
    phase[0] = name
    t0 = time.perf_counter()
    stages = []
    for _ in range(calls):
        if name.startswith("serial"):
            d.process_device(iq, n, bits, nbits)
            stages.append(d.stage_times())
        else:
            d.process_device_async(iq, n, bits, nbits)
    if name == "pipelined":
        d.pipeline_wait()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    phase[0] = "idle"
    e1 = [energy(h) for h in handles]
    results[name] = (dt, [b - a for a, b in zip(e0, e1)], stages)
    time.sleep(0.3)
stop.set()
th.join()

# the busy card: largest energy over the run
busy = max(range(len(handles)), key=lambda i: sum(r[1][i] for r in results.values()))
os.makedirs("gpurun_out", exist_ok=True)
with open(f"gpurun_out/power_{key}.csv", "w") as f:
    f.write("t_s,phase,watts,gfx_mhz\n")
    for t, ph, row in samples:
        f.write(f"{t - samples[0][0]:.4f},{ph},{row[busy][0]:.1f},{row[busy][1]:.0f}\n")
print(f"config {key}: S={S} sps={sps} T={span * sps + 1} calls={calls} busy card {busy} of {len(handles)}")
for name, (dt, de, stages) in results.items():
    pts = [r[busy] for t, ph, r in samples if ph == name]
    ws = sorted(w for w, _ in pts)
    mh = sorted(c for _, c in pts)
    q = lambda v, f: v[min(len(v) - 1, int(f * len(v)))] if v else float("nan")   # noqa: E731
    st = ""
    if stages:
        keys = [k for k in stages[0] if stages[0][k] > 0.01]
        st = " ".join(f"{k}={sum(s[k] for s in stages) / len(stages):.1f}ms" for k in keys)
    print(f"{name:9s} {1e3 * dt / calls:7.2f} ms/call  energy {de[busy] / calls:6.2f} J/call "
          f"({de[busy] / dt:6.0f} W avg)  samples {len(pts)}: W p10/p50/p90 {q(ws, .1):.0f}/{q(ws, .5):.0f}/"
          f"{q(ws, .9):.0f}  MHz p10/p50/p90 {q(mh, .1):.0f}/{q(mh, .5):.0f}/{q(mh, .9):.0f}  {st}", flush=True)
try:
    cap = amdsmi.amdsmi_get_power_info(handles[busy]).get("power_limit")
    print("power_limit", cap)
except Exception as exc:   # noqa: BLE001
    print("power_limit n/a", exc)
amdsmi.amdsmi_shut_down()
