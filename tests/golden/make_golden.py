"""Generate the committed golden fixtures (SURVEY.md §8c "Fixtures").

The reference ships no golden vectors and its C# cannot run here (no .NET), so
the fixtures are produced by the CPU oracle (oracle/, the C restatement) and
cross-checked, in tests/test_golden.py, against the independent numpy model
(tests/refmodel.py).  Inputs are stored next to the outputs so the GPU tests
need neither the generator nor /root/reference.

    python tests/golden/make_golden.py          # rewrites tests/golden/*.npz

Fixtures
  tad_literal.npz  testAtDataLevel.cs:15-58 literally: fs 10 MS/s, sps 2,
                   rrcSpan 10 (21 taps), alpha 0.4f, the 64-bit TSC, frames of
                   "MESSAGE_START" + payload + "MESSAGE_STOP" through two
                   +-1 ppm 100 MHz LOs (seeded), 15 frames, one persistent
                   demodulator per API.
  tad_sps8.npz     BASELINE configs[0]: the same procedure at sps 8 / 65 taps on
                   10 000 random symbols, one DeModulate call; MF output (first
                   8192 samples), bits, rotated symbols (portable and glibc trig).
  impaired.npz     4 streams x 16384 samples, +-5 kHz CFO, 4-tap multipath,
                   20 dB AWGN; bits + symbols with the FLL off and on, fed in
                   two ragged calls per stream.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import common as K  # noqa: E402
import oracle as O  # noqa: E402

START, STOP = "MESSAGE_START", "MESSAGE_STOP"


def bitstr_to_u8(s: str) -> np.ndarray:
    return np.frombuffer(s.encode(), np.uint8) - ord("0")


def concat(parts, dtype):
    lens = np.array([len(p) for p in parts], np.int64)
    flat = np.concatenate([np.asarray(p, dtype) for p in parts]) if parts else np.zeros(0, dtype)
    return flat, lens


def tad_literal():
    sps, span = 2, 10
    fs, rs = K.FS, K.FS // sps
    tx = O.OracleNCO(100e6, fs, 1, 0, seed=11)
    rx = O.OracleNCO(100e6, fs, 1, 0, seed=22)
    d_text = O.OracleDemod(fs, rs, K.ALPHA, span, tsc=K.TSC)
    d_bits = O.OracleDemod(fs, rs, K.ALPHA, span, tsc=K.TSC)
    frames, texts, bits, raw, syms = [], [], [], [], []
    for _ in range(15):
        sig = O.modulate_text_utf8(fs, rs, K.PAYLOAD, START, STOP, rrc_alpha=K.ALPHA,
                                   rrc_span=span, tsc=K.TSC)
        sig = O.apply_lo_pair(tx, rx, sig)
        frames.append(sig)
        texts.append(np.frombuffer(d_text.DeModulateTextUtf8(sig, START, STOP).encode("utf-8"), np.uint8))
    # the bits API on a third instance: raw bits + symbols, and the TSC-stripped string
    d_raw = O.OracleDemod(fs, rs, K.ALPHA, span, tsc=K.TSC)
    for sig in frames:
        bits.append(bitstr_to_u8(d_bits.DeModulate(sig)))
        b, s, _ = d_raw.demodulate_ex(sig)
        raw.append(bitstr_to_u8(b))
        syms.append(s)
    f, fl = concat(frames, np.float32)
    t, tl = concat(texts, np.uint8)
    b, bl = concat(bits, np.uint8)
    r, rl = concat(raw, np.uint8)
    s, sl = concat(syms, np.float32)
    np.savez_compressed(os.path.join(HERE, "tad_literal.npz"), sps=sps, span=span,
                        iq=f, iq_len=fl, text=t, text_len=tl, bits=b, bits_len=bl,
                        raw_bits=r, raw_bits_len=rl, syms=s, syms_len=sl)


def tad_sps8():
    sps, span = 8, 8
    iq = K.stream_signal(7, sps=sps, span=span, n_bits=20000)
    dm = K.oracle_for(sps, span)
    b, s, _ = dm.demodulate_ex(iq)
    dl = K.oracle_for(sps, span, trig=O.TRIG_LIBM)
    bl, sl, _ = dl.demodulate_ex(iq)
    assert bl == b
    mf = O.oracle_fir(np.stack([dm.rrc_f32(), np.zeros_like(dm.rrc_f32())], 1).reshape(-1), iq)
    np.savez_compressed(os.path.join(HERE, "tad_sps8.npz"), sps=sps, span=span, iq=iq,
                        mf_head=mf[: 2 * 8192], bits=bitstr_to_u8(b), syms=s, syms_libm=sl)


def impaired():
    sps, span, S, n = 8, 8, 4, 16384
    rng = np.random.default_rng(5)
    sigs = [K.stream_signal(100 + s, sps=sps, span=span, n_bits=2 * n // sps + 64, snr_db=20,
                            cfo_hz=float(rng.uniform(-5e3, 5e3)), multipath=True)[: 2 * n]
            for s in range(S)]
    iq = np.stack(sigs)
    split = np.array([5000 + 1111 * s for s in range(S)], np.int64)   # ragged first call
    out = {}
    for tag, fll in (("off", False), ("on", True)):
        bits, blen, syms, slen = [], [], [], []
        for s in range(S):
            dm = K.oracle_for(sps, span, enable_fll=fll)
            for a, z in ((0, split[s]), (split[s], n)):
                b, y, _ = dm.demodulate_ex(iq[s, 2 * a: 2 * z])
                bits.append(bitstr_to_u8(b))
                syms.append(y)
        out[f"bits_{tag}"], out[f"bits_{tag}_len"] = concat(bits, np.uint8)
        out[f"syms_{tag}"], out[f"syms_{tag}_len"] = concat(syms, np.float32)
    np.savez_compressed(os.path.join(HERE, "impaired.npz"), sps=sps, span=span, iq=iq,
                        split=split, **out)


if __name__ == "__main__":
    tad_literal()
    tad_sps8()
    impaired()
    for f in sorted(os.listdir(HERE)):
        print(f, os.path.getsize(os.path.join(HERE, f)))
