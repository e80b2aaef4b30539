"""Diagnostic: per-call loop-kernel time and loop-state statistics over a
sustained run of consecutive DeModulate calls on the same synthetic batch.

Reports, after each call, how many streams have |theta| > 1e6 (round 1's Costas fast-sincos range) and > 2^40 (the current range), |freq| > pi (the single +-2pi wrap can
no longer bound theta), a non-finite M&M time, or a sticky error flag."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qpsk-modulator-demodulator_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--calls", type=int, default=12)
    ap.add_argument("--streams", type=int, default=0)
    a = ap.parse_args()
    import torch
    import bench as B
    import qpsk_amd as Q
    cfg = B.CONFIGS[a.config]
    S = a.streams or cfg["streams"]
    n = 1 << 20
    sps, span = cfg["sps"], cfg["span"]
    iq, _ = Q.synth_generate(S, n, B.FS, B.FS // sps, rrc_alpha=B.ALPHA, rrc_span=span,
                             seed=0x5159534B, lo_ppm=1.0,
                             cfo_hz=5000.0 if cfg["impaired"] else 0.0, multipath=cfg["impaired"],
                             esn0_db=20.0 if cfg["impaired"] else None)
    d = Q.BatchDemodulator(S, Q.params(B.FS, B.FS // sps, B.ALPHA, span, enable_fll=cfg["fll"],
                                       max_samples_per_call=n))
    ms = d.max_symbols(n)
    bits = torch.zeros((S, (2 * ms + 7) // 8 + 64), dtype=torch.uint8, device="cuda")
    nb = torch.zeros(S, dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    d.set_stream(st.cuda_stream)
    for c in range(a.calls):
        d.enable_timing(True)
        d.process_device(iq, n, bits, nb)
        torch.cuda.synchronize()
        t = d.stage_times()
        d.enable_timing(False)
        s = d.stream_states()
        th, fr = np.abs(s["theta"]), np.abs(s["freq"])
        rec = {"call": c, "fll_ms": round(t.get("fll", 0.0), 2), "fir_ms": round(t["fir"], 2), "loop_ms": round(t["loop"], 2),
               "theta_gt_1e6": int((th > 1e6).sum()), "theta_gt_2p40": int((th > 2.0 ** 40).sum()),
               "theta_max": float(th.max()),
               "freq_gt_pi": int((fr > np.pi).sum()), "freq_max": float(fr.max()),
               "mu_nonfinite": int((~np.isfinite(s["mu"])).sum()),
               "error_flags": int((s["error"] != 0).sum()),
               "waves_with_huge": int(len(set((np.nonzero(th > 1e6)[0] // 32).tolist()))),
               "nbits_min": int(nb.min()), "nbits_max": int(nb.max())}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
