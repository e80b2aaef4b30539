"""Golden fixtures (tests/golden/, written by tests/golden/make_golden.py).

CPU: the oracle reproduces every fixture, and the independent numpy model
(refmodel.py) reproduces the bits, symbols and matched-filter output of the
two testAtDataLevel-style fixtures -- this pins the oracle against a second
restatement, since the C# reference cannot run here (DESIGN.md "Parity").

GPU: the HIP path through the C ABI reproduces every fixture bit for bit
(bits, rotated symbols, framer payloads), with no oracle in the loop.
"""
import os

import numpy as np
import pytest

import common as K
import oracle as O
import refmodel as RM

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
START, STOP = "MESSAGE_START", "MESSAGE_STOP"


def load(name):
    return np.load(os.path.join(GOLD, name))


def split(flat, lens):
    out, o = [], 0
    for n in lens:
        out.append(flat[o: o + n])
        o += n
    return out


def bits_str(u8):
    return (np.asarray(u8, np.uint8) + ord("0")).tobytes().decode()


# ---------------------------------------------------------------- CPU

def test_oracle_reproduces_tad_literal():
    z = load("tad_literal.npz")
    sps, span = int(z["sps"]), int(z["span"])
    frames = split(z["iq"], z["iq_len"])
    texts = split(z["text"], z["text_len"])
    bits = split(z["bits"], z["bits_len"])
    raw = split(z["raw_bits"], z["raw_bits_len"])
    syms = split(z["syms"], z["syms_len"])
    dt = O.OracleDemod(K.FS, K.FS // sps, K.ALPHA, span, tsc=K.TSC)
    db = O.OracleDemod(K.FS, K.FS // sps, K.ALPHA, span, tsc=K.TSC)
    dr = O.OracleDemod(K.FS, K.FS // sps, K.ALPHA, span, tsc=K.TSC)
    ok = 0
    for f, t, b, r, s in zip(frames, texts, bits, raw, syms):
        got = dt.DeModulateTextUtf8(f, START, STOP)
        assert got.encode("utf-8") == t.tobytes()
        ok += K.PAYLOAD in got
        assert db.DeModulate(f) == bits_str(b)
        rb, rs, _ = dr.demodulate_ex(f)
        assert rb == bits_str(r)
        assert np.array_equal(rs, s)
    # the reference's own pass criterion (testAtDataLevel.cs:46), 14 of 15 frames
    assert ok >= 14


def test_refmodel_reproduces_tad_literal():
    z = load("tad_literal.npz")
    sps, span = int(z["sps"]), int(z["span"])
    m = RM.RefDemod(K.FS, K.FS // sps, K.ALPHA, span)
    for f, r, s in zip(split(z["iq"], z["iq_len"]), split(z["raw_bits"], z["raw_bits_len"]),
                       split(z["syms"], z["syms_len"])):
        b, rot, _ = m.demodulate(f)
        assert b == bits_str(r)
        assert np.array_equal(rot, s)


def test_oracle_and_refmodel_reproduce_tad_sps8():
    z = load("tad_sps8.npz")
    sps, span = int(z["sps"]), int(z["span"])
    iq = z["iq"]
    b, s, _ = K.oracle_for(sps, span).demodulate_ex(iq)
    assert b == bits_str(z["bits"]) and K.bitwise_equal(s, z["syms"])
    bl, sl, _ = K.oracle_for(sps, span, trig=O.TRIG_LIBM).demodulate_ex(iq)
    assert bl == b and K.bitwise_equal(sl, z["syms_libm"])
    assert np.max(np.abs(sl - s)) <= 1e-5
    m = RM.RefDemod(K.FS, K.FS // sps, K.ALPHA, span)
    rb, rot, mf = m.demodulate(iq)
    assert rb == b
    assert np.array_equal(rot, s)
    assert K.bitwise_equal(mf[: z["mf_head"].size], z["mf_head"])


def test_oracle_reproduces_impaired():
    z = load("impaired.npz")
    sps, span, iq, cut = int(z["sps"]), int(z["span"]), z["iq"], z["split"]
    n = iq.shape[1] // 2
    for tag, fll in (("off", False), ("on", True)):
        bits = split(z[f"bits_{tag}"], z[f"bits_{tag}_len"])
        syms = split(z[f"syms_{tag}"], z[f"syms_{tag}_len"])
        i = 0
        for s in range(iq.shape[0]):
            dm = K.oracle_for(sps, span, enable_fll=fll)
            for a, e in ((0, cut[s]), (cut[s], n)):
                b, y, _ = dm.demodulate_ex(iq[s, 2 * a: 2 * e])
                assert b == bits_str(bits[i]) and K.bitwise_equal(y, syms[i])
                i += 1


# ---------------------------------------------------------------- GPU

@pytest.fixture(scope="module")
def Q():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need an MI355X")
    import qpsk_amd
    return qpsk_amd


@pytest.mark.gpu
def test_gpu_tad_literal_mirror(Q):
    """testAtDataLevel.cs:15-58 through the single-stream mirror class."""
    z = load("tad_literal.npz")
    sps, span = int(z["sps"]), int(z["span"])
    g_text = Q.QPSKDeModulator(K.FS, K.FS // sps, K.ALPHA, span, tsc=K.TSC)
    g_bits = Q.QPSKDeModulator(K.FS, K.FS // sps, K.ALPHA, span, tsc=K.TSC)
    for f, t, b in zip(split(z["iq"], z["iq_len"]), split(z["text"], z["text_len"]),
                       split(z["bits"], z["bits_len"])):
        assert g_text.DeModulateTextUtf8(f, START, STOP).encode("utf-8") == t.tobytes()
        assert g_bits.DeModulate(f) == bits_str(b)


@pytest.mark.gpu
def test_gpu_tad_literal_raw_symbols(Q):
    z = load("tad_literal.npz")
    sps, span = int(z["sps"]), int(z["span"])
    frames = split(z["iq"], z["iq_len"])
    b = Q.BatchDemodulator(1, Q.params(K.FS, K.FS // sps, K.ALPHA, span,
                                       max_samples_per_call=int(z["iq_len"].max()) // 2 + 8))
    for f, r, s in zip(frames, split(z["raw_bits"], z["raw_bits_len"]), split(z["syms"], z["syms_len"])):
        bits, nb, syms, ns = b.process(f[None, :], want_syms=True)
        assert Q.unpack_bits(bits[0], int(nb[0])) == bits_str(r)
        assert K.bitwise_equal(syms[0, : 2 * int(ns[0])], s)
    b.close()


@pytest.mark.gpu
def test_gpu_tad_sps8(Q):
    z = load("tad_sps8.npz")
    sps, span, iq = int(z["sps"]), int(z["span"]), z["iq"]
    b = Q.BatchDemodulator(1, Q.params(K.FS, K.FS // sps, K.ALPHA, span, max_samples_per_call=iq.size // 2))
    bits, nb, syms, ns = b.process(iq[None, :], want_syms=True)
    assert Q.unpack_bits(bits[0], int(nb[0])) == bits_str(z["bits"])
    assert K.bitwise_equal(syms[0, : 2 * int(ns[0])], z["syms"])
    assert np.max(np.abs(syms[0, : 2 * int(ns[0])] - z["syms_libm"])) <= 1e-5
    b.close()
    # the Costas NCO on glibc's own sin/cos: the libm fixture, bit for bit
    b = Q.BatchDemodulator(1, Q.params(K.FS, K.FS // sps, K.ALPHA, span, max_samples_per_call=iq.size // 2,
                                       costas_trig=1))
    bits, nb, syms, ns = b.process(iq[None, :], want_syms=True)
    assert Q.unpack_bits(bits[0], int(nb[0])) == bits_str(z["bits"])
    assert K.bitwise_equal(syms[0, : 2 * int(ns[0])], z["syms_libm"])
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("tag,fll", [("off", False), ("on", True)])
def test_gpu_impaired_ragged(Q, tag, fll):
    z = load("impaired.npz")
    sps, span, iq, cut = int(z["sps"]), int(z["span"]), z["iq"], z["split"]
    S, n = iq.shape[0], iq.shape[1] // 2
    bits = split(z[f"bits_{tag}"], z[f"bits_{tag}_len"])
    syms = split(z[f"syms_{tag}"], z[f"syms_{tag}_len"])
    b = Q.BatchDemodulator(S, Q.params(K.FS, K.FS // sps, K.ALPHA, span, enable_fll=fll,
                                       max_samples_per_call=n))
    for call in range(2):
        lens = cut if call == 0 else n - cut
        m = int(lens.max())
        x = np.zeros((S, 2 * m), np.float32)
        for s in range(S):
            a = 0 if call == 0 else cut[s]
            x[s, : 2 * lens[s]] = iq[s, 2 * a: 2 * (a + lens[s])]
        gb, nb, gs, ns = b.process(x, lengths=lens, want_syms=True)
        for s in range(S):
            i = 2 * s + call
            assert Q.unpack_bits(gb[s], int(nb[s])) == bits_str(bits[i]), f"stream {s} call {call}"
            assert K.bitwise_equal(gs[s, : 2 * int(ns[s])], syms[i]), f"stream {s} call {call}"
    b.close()
