#!/usr/bin/env python3
"""tools/ber_slips.py -- where the clean-channel bit errors of the bench come from.

The bench's clean configs (C2/C3/C4: differential QPSK through a +-1 ppm
100 MHz LO pair, no noise) report a nonzero BER with symbol slips and lost
windows, and the CPU oracle's rows give the same counts (bench.py `ber_cpu`).
This script runs only the CPU oracle (glibc trig, the libm restatement of the
reference) on inputs synthesised here with the bench's own recipe
(qpsk_synth.hip restated in numpy: splitmix64 payloads and carrier, direct RRC
pulse shaping), and separates the candidate causes:

  E1  a static carrier phase phi0, no frequency offset: slips vs phi0
  E2  a frequency offset f, random phi0: slips vs |f|
  E3  the C2 bench streams themselves (their f and phi0 from the synth's RNG),
      as synthesised, and with the carrier removed by a genie before the chain
  E4  the timing loop alone (MF -> MuellerMuller) at a static phase

Usage: python tools/ber_slips.py [--streams 32] [--out profiles/r05_ber_slips.txt]
"""
import argparse
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
import oracle as O  # noqa: E402

FS = 10_000_000
ALPHA = 0.4000000059604645
SEED = 0x5159534B
M64 = (1 << 64) - 1


def splitmix64(st):
    st = (st + 0x9E3779B97F4A7C15) & M64
    z = st
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return st, z ^ (z >> 31)


def u01(v):
    return (v >> 11) * 2.0 ** -53


def carrier(gs, lo_ppm=1.0, lo_hz=100e6):
    """(frequency offset Hz, initial phase rad) of global stream gs
    (qpsk_synth.hip:119-126)."""
    rs = SEED ^ ((0xC0FFEE123 + gs * 0xD1B54A32D192ED03) & M64)
    rs, a = splitmix64(rs)
    rs, b = splitmix64(rs)
    rs, c = splitmix64(rs)
    f = lo_hz * ((2.0 * u01(a) - 1.0) - (2.0 * u01(b) - 1.0)) * lo_ppm * 1e-6
    return f, 2.0 * np.pi * u01(c)


def payload(gs, nsym):
    """Differential quadrant indices and packed payload bits of stream gs
    (qpsk_synth.hip:65-98)."""
    rng = SEED ^ ((0x5159534B + gs * 0x9E3779B97F4A7C15) & M64)
    dib = np.empty(nsym, np.uint8)
    for w in range((nsym + 31) // 32):
        rng, word = splitmix64(rng)
        k = min(32, nsym - 32 * w)
        sh = np.arange(62, 62 - 2 * k, -2, dtype=np.uint64)
        dib[32 * w: 32 * w + k] = ((np.uint64(word) >> sh) & np.uint64(3)).astype(np.uint8)
    rot = np.array([0, 1, 3, 2], np.uint8)[dib]
    quad = (np.cumsum(rot, dtype=np.int64) & 3).astype(np.uint8)
    bits = np.unpackbits(dib[:, None], axis=1)[:, 6:].reshape(-1)
    return quad, np.packbits(bits)


def synth(gs, n, sps, span, f=None, phi0=None):
    """One clean stream as the bench synthesises it (float32 interleaved) and
    its packed payload bits; f / phi0 override the carrier (None: the
    stream's own)."""
    h = O.rrc_taps(span, ALPHA, FS, FS // sps).astype(np.float32).astype(np.float64)
    T = h.size
    mid = (T - 1) // 2
    nsym = (n + mid) // sps + 2
    quad, bits = payload(gs, nsym)
    c = 0.70710678118654752440
    sym = (np.array([c, -c, -c, c]) + 1j * np.array([c, c, -c, -c]))[quad]
    up = np.zeros(nsym * sps, np.complex128)
    up[::sps] = sym
    y = np.convolve(up, h)[mid: mid + n]
    f0, p0 = carrier(gs)
    f = f0 if f is None else f
    p0 = p0 if phi0 is None else phi0
    if f != 0.0 or p0 != 0.0:
        y = y * np.exp(1j * (2.0 * np.pi * f * np.arange(n) / FS + p0))
    return np.stack([y.real, y.imag], 1).astype(np.float32).reshape(-1), bits


def ber(rows, nbits, tx):
    import bench
    return bench.ber_after_lock(rows, nbits, tx, rows.shape[0])


def demod(iq2d, sps, span, threads=8):
    bits, nb, _, _ = O.demod_batch_packed(iq2d, FS, FS // sps, n_threads=threads, rrc_alpha=ALPHA,
                                          rrc_span=span, trig=O.TRIG_LIBM)
    return bits, nb


def per_stream(iqs, txs, sps, span):
    bits, nb = demod(np.stack(iqs), sps, span)
    out = []
    for s in range(len(iqs)):
        out.append(ber(bits[s: s + 1], nb[s: s + 1], txs[s][None, :]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=32)
    ap.add_argument("--samples", type=int, default=1 << 20)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05_ber_slips.txt"))
    a = ap.parse_args()
    sps, span, n = 8, 8, a.samples
    lines = []

    def log(s=""):
        print(s, flush=True)
        lines.append(s)

    t0 = time.time()
    log(f"# tools/ber_slips.py: CPU oracle (glibc trig), sps {sps}, {span * sps + 1} taps, "
        f"{n} samples per stream, clean channel (no noise); BER counter = bench.ber_after_lock")
    log("# columns: bit_errors bits lost_windows symbol_slips")

    log("\n## E1: static carrier phase, no frequency offset (stream 0's payload)")
    phis = np.linspace(0.0, np.pi / 2, 17)
    with ThreadPoolExecutor(4) as ex:
        sig = list(ex.map(lambda p: synth(0, n, sps, span, f=0.0, phi0=p), phis))
    res = per_stream([s[0] for s in sig], [s[1] for s in sig], sps, span)
    for p, r in zip(phis, res):
        log(f"phi0 {np.degrees(p):6.2f} deg: {r}")

    log("\n## E2: frequency offset f, stream 0's payload, phi0 = 0.3 rad")
    fs_ = [0.0, 10.0, 25.0, 50.0, 100.0, 150.0, 200.0]
    with ThreadPoolExecutor(4) as ex:
        sig = list(ex.map(lambda f: synth(0, n, sps, span, f=f, phi0=0.3), fs_))
    res = per_stream([s[0] for s in sig], [s[1] for s in sig], sps, span)
    for f, r in zip(fs_, res):
        turns = f * n / FS
        log(f"f {f:6.1f} Hz ({turns:5.2f} carrier turns, {4 * turns:5.1f} passes through a 45-deg "
            f"offset): {r}")

    log("\n## E4: the timing loop alone (MF -> MuellerMuller, the reference's first loop), "
        "static phase, stream 0's payload")
    log("# symbols out and the mean |x|^2 of the last half (~1 = sampling on the symbol peaks)")
    dm = O.OracleDemod(FS, FS // sps, ALPHA, span)
    g = dm.gains()
    taps = dm.rrc_f32()
    tiq = np.stack([taps, np.zeros_like(taps)], 1).reshape(-1)
    for p in (0.0, np.pi / 8, 3 * np.pi / 16, np.pi / 4):
        x, _ = synth(0, n, sps, span, f=0.0, phi0=p)
        mf = O.oracle_fir(tiq, x)
        mm = O.OracleMM(g["mm_sps"], g["kp"], g["ki"])
        sy = mm.process(mf).reshape(-1, 2)
        half = sy[sy.shape[0] // 2:]
        pw = float(np.mean(half[:, 0].astype(np.float64) ** 2 + half[:, 1].astype(np.float64) ** 2))
        log(f"phi0 {np.degrees(p):6.2f} deg: {sy.shape[0]} symbols (n/sps = {n // sps}), "
            f"mean |x|^2 {pw:.4f}")

    log(f"\n## E3: the bench's C2 streams 0..{a.streams - 1} (own f, phi0): as synthesised | "
        "carrier removed before the chain")
    ids = list(range(a.streams))
    with ThreadPoolExecutor(4) as ex:
        sig = list(ex.map(lambda g: synth(g, n, sps, span), ids))
        gen = list(ex.map(lambda g: synth(g, n, sps, span, f=0.0, phi0=0.0), ids))
    res = per_stream([s[0] for s in sig], [s[1] for s in sig], sps, span)
    res0 = per_stream([s[0] for s in gen], [s[1] for s in gen], sps, span)
    tot = np.zeros(4, np.int64)
    tot0 = np.zeros(4, np.int64)
    rows = []
    for g, r, r0 in zip(ids, res, res0):
        f, p = carrier(g)
        rows.append((abs(f), g, f, p, r, r0))
        tot += r
        tot0 += r0
    for _, g, f, p, r, r0 in sorted(rows):
        log(f"stream {g:3d}: f {f:8.2f} Hz phi0 {np.degrees(p):6.1f} deg: {r} | {r0}")
    log(f"total: {tuple(int(v) for v in tot)} | {tuple(int(v) for v in tot0)}")
    fa = np.array([r[0] for r in rows])
    sl = np.array([r[4][3] + r[4][2] for r in rows], np.float64)
    if sl.std() > 0:
        log(f"corr(|f|, slips + lost windows) = {np.corrcoef(fa, sl)[0, 1]:.3f}")
    log(f"\n# {time.time() - t0:.1f} s")
    if a.out:
        with open(a.out, "w") as fh:
            fh.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
