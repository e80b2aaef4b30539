"""Shared signal helpers for the tests (seeded, small).

Inputs follow the reference's own test procedure (testAtDataLevel.cs:15-58):
QPSKModulator output (oracle restatement) through a pair of ±1 ppm 100 MHz
LOs, optionally with AWGN / carrier offset / multipath for impaired cases.
"""
import numpy as np

import oracle as O

FS = 10_000_000
ALPHA = float(np.float32(0.4))                      # testAtDataLevel.cs:18 (float)
TSC = "11001010011101100100100110101100" + "01110100111001011010001101101001"   # :20-22
PAYLOAD = "The Quick Brown fox jump yes yes man good!"                          # :35

# (sps, rrc span) -> taps = span*sps+1: 65 (BASELINE C1/C2), 129 (C3), 21 (literal tAD)
CONFIGS = [(8, 8), (4, 32), (2, 10)]


def random_bits(rng, n):
    return "".join(rng.choice(["0", "1"], n))


def stream_signal(seed, sps=8, span=8, n_bits=2000, snr_db=None, cfo_hz=0.0, multipath=False,
                  differential=True, lo=True):
    """One clean (or impaired) stream as interleaved float32."""
    rng = np.random.default_rng(seed)
    rs = FS // sps
    sig = O.modulate(FS, rs, random_bits(rng, n_bits), rrc_alpha=ALPHA, rrc_span=span,
                     differential=differential)
    if lo:
        tx = O.OracleNCO(100e6, FS, 1, 0, seed=1000 + seed)
        rx = O.OracleNCO(100e6, FS, 1, 0, seed=2000 + seed)
        sig = O.apply_lo_pair(tx, rx, sig)
    z = sig.reshape(-1, 2).astype(np.float64)
    c = z[:, 0] + 1j * z[:, 1]
    if multipath:
        h = np.array([1, 0.25 * np.exp(0.7j), 0.1 * np.exp(-1.9j), 0.05])
        c = np.convolve(c, h)[: c.size]
    if cfo_hz:
        c = c * np.exp(2j * np.pi * cfo_hz / FS * np.arange(c.size) + 1j * rng.uniform(0, 6.28))
    if snr_db is not None:
        p = np.mean(np.abs(c) ** 2)
        s = np.sqrt(p / 10 ** (snr_db / 10) / 2)
        c = c + s * (rng.standard_normal(c.size) + 1j * rng.standard_normal(c.size))
    return np.stack([c.real, c.imag], 1).astype(np.float32).reshape(-1)


def batch_signals(n_streams, seed0=0, **kw):
    sigs = [stream_signal(seed0 + s, **kw) for s in range(n_streams)]
    n = min(x.size for x in sigs)
    return np.stack([x[:n] for x in sigs])


def oracle_for(sps, span, **kw):
    return O.OracleDemod(FS, FS // sps, ALPHA, span, **kw)


def bitwise_equal(a, b, nan_any_payload=False):
    """Exact float parity: same dtype, shape and bit patterns, so -0 vs +0 and
    NaN payloads count (np.array_equal treats +-0 as equal and never matches a
    NaN).  nan_any_payload: NaN must meet NaN at the same positions, but its
    payload may differ (the default NaN of an invalid operation is 0xFFC00000 on
    x86, where the oracle runs, and 0x7FC00000 on gfx950); every other value
    still compares bit for bit."""
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    if a.dtype != b.dtype or a.shape != b.shape:
        return False
    if a.dtype.kind != "f":
        return bool(np.array_equal(a, b))
    u = {2: np.uint16, 4: np.uint32, 8: np.uint64}[a.dtype.itemsize]
    if nan_any_payload:
        na, nb = np.isnan(a), np.isnan(b)
        if not np.array_equal(na, nb):
            return False
        return bool(np.array_equal(a[~na].view(u), b[~nb].view(u)))
    return bool(np.array_equal(a.view(u), b.view(u)))
