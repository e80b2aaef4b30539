"""tools/overlap_probe.py -- time the C2 matched filter (serial DeModulate calls)
while a stand-in for the loop kernel (tools/overlap_probe.hip) occupies 8 CUs on
another stream.  Diagnostic only (pipelined-call interference)."""
import ctypes as C, os, sys, time
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "qpsk-modulator-demodulator_amd"))
import qpsk_amd as Q

so = C.CDLL(os.path.join(os.path.dirname(__file__), "..", "qpsk-modulator-demodulator_amd", "_build", "overlap_probe.so"))
S, n = 256, 1 << 20
p = Q.params(10_000_000, 1_250_000, rrc_alpha=0.4, rrc_span=8)
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
            so.launch_sleeper(C.c_void_p(sb.cuda_stream), C.c_longlong(6_000_000), lds, busy,
                              C.c_void_p(sink.data_ptr()), 8)
            time.sleep(0.002)
        with torch.cuda.stream(sa):
            d.process_device(iq, n, bits, nb)
        sa.synchronize()
        out.append(d.stage_times()["fir"])
        torch.cuda.synchronize()
    return out

for name, kind in [("alone", None), ("sleep_lds", (146944, 0)), ("sleep_nolds", (0, 0)),
                   ("busy_lds", (146944, 1)), ("alone2", None)]:
    print(name, " ".join(f"{v:.3f}" for v in fir_ms(kind)), flush=True)
