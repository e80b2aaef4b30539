"""tools/overlap_probe.py -- time the matched filter (serial DeModulate calls)
while a stand-in for the loop kernel (tools/overlap_probe.hip) occupies WGS CUs
on another stream.  Diagnostic only (pipelined-call interference).
Usage: overlap_probe.py [S sps span wgs lds_bytes]  (default C2: 256 8 8 8 146944)"""
import ctypes as C, os, sys, time
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "qpsk-modulator-demodulator_amd"))
import qpsk_amd as Q

so = C.CDLL(os.path.join(os.path.dirname(__file__), "..", "qpsk-modulator-demodulator_amd", "_build", "overlap_probe.so"))
S, SPS, SPAN, WGS, LDS = (int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (256, 8, 8, 8, 146944)))
n = 1 << 20
p = Q.params(10_000_000, 10_000_000 // SPS, rrc_alpha=0.4, rrc_span=SPAN)
d = Q.BatchDemodulator(S, p)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
d.set_stream(sa.cuda_stream)
d.enable_timing(True)
iq = torch.randn(S, 2 * n, device="cuda")
cap = d.max_symbols(n)
bits = torch.zeros(S, (2 * cap + 7) // 8 + 8, dtype=torch.uint8, device="cuda")
nb = torch.zeros(S, dtype=torch.int64, device="cuda")
sink = torch.zeros(256, device="cuda")

def fir_ms(kind):
    out = []
    for _ in range(4):
        torch.cuda.synchronize()
        if kind is not None:
            lds, busy = kind
            so.launch_sleeper(C.c_void_p(sb.cuda_stream), C.c_longlong(6_000_000 if S <= 256 else 20_000_000),
                              lds, busy, C.c_void_p(sink.data_ptr()), WGS)
            time.sleep(0.002)
        with torch.cuda.stream(sa):
            d.process_device(iq, n, bits, nb)
        sa.synchronize()
        out.append(d.stage_times()["fir"])
        torch.cuda.synchronize()
    return out

for name, kind in [("alone", None), ("sleep_lds", (LDS, 0)), ("sleep_nolds", (0, 0)),
                   ("busy_lds", (LDS, 1)), ("busy_nolds", (0, 1)), ("alone2", None)]:
    print(name, " ".join(f"{v:.3f}" for v in fir_ms(kind)), flush=True)
