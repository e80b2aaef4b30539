"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar (DESIGN.md "Parity"): with the portable trig the oracle and the GPU run
the same IEEE operation sequence, so bits AND rotated symbols must be
bit-identical; against the glibc-trig oracle (what .NET-on-Linux calls) bits
must be identical and symbols within 1e-5 absolute.
"""
import numpy as np
import pytest

import common as K
import oracle as O
import qpsk_amd as Q

pytestmark = pytest.mark.gpu

SYM_TOL = 1e-5   # constellation tolerance vs the libm-trig oracle


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need an MI355X")
    yield


def oracle_run(iq2d, calls, sps, span, mode=None, **kw):
    """Per-stream oracle instances fed the same call sequence.
    calls: list of per-call [S] lengths (complex samples); mode per call."""
    S = iq2d.shape[0]
    dms = [K.oracle_for(sps, span, **kw) for _ in range(S)]
    pos = np.zeros(S, dtype=np.int64)
    out = []
    for ci, lens in enumerate(calls):
        m = mode[ci] if mode else Q.MODE_DEMODULATE
        res = []
        for s in range(S):
            x = iq2d[s, 2 * pos[s]: 2 * (pos[s] + lens[s])]
            if m == Q.MODE_DEMODULATE:
                bits, syms, _ = dms[s].demodulate_ex(x)
                res.append((bits, syms))
            else:
                res.append(("", dms[s].deModulateConstellation(x)))
            pos[s] += lens[s]
        out.append(res)
    return out


def gpu_run(iq2d, calls, sps, span, mode=None, want_syms=True, **kw):
    """want_syms=False runs the bits-only kernel (decisions-only Costas ->
    decode slots); its rows carry bits and None for the symbols."""
    S = iq2d.shape[0]
    p = Q.params(K.FS, K.FS // sps, K.ALPHA, span, max_samples_per_call=max(max(c) for c in calls) + 8, **kw)
    b = Q.BatchDemodulator(S, p)
    pos = np.zeros(S, dtype=np.int64)
    out = []
    for ci, lens in enumerate(calls):
        m = mode[ci] if mode else Q.MODE_DEMODULATE
        n = int(max(lens))
        x = np.zeros((S, 2 * max(n, 1)), np.float32)
        for s in range(S):
            x[s, : 2 * lens[s]] = iq2d[s, 2 * pos[s]: 2 * (pos[s] + lens[s])]
        uniform = all(l == lens[0] for l in lens)
        bits, nb, syms, ns = b.process(x[:, : 2 * n] if n else x[:, :0], mode=m,
                                       lengths=None if uniform else np.array(lens), want_syms=want_syms)
        res = []
        for s in range(S):
            bs = Q.unpack_bits(bits[s], int(nb[s])) if m == Q.MODE_DEMODULATE else ""
            res.append((bs, syms[s, : 2 * int(ns[s])].copy() if want_syms else None))
        pos += np.array(lens)
        out.append(res)
    b.close()
    return out


def assert_same(a, b, exact=True):
    for ci, (ra, rb) in enumerate(zip(a, b)):
        for s, ((ba, sa), (bb, sb)) in enumerate(zip(ra, rb)):
            assert ba == bb, f"call {ci} stream {s}: bits differ ({len(ba)} vs {len(bb)})"
            if sa is None or sb is None:
                continue
            assert sa.shape == sb.shape, f"call {ci} stream {s}: symbol count"
            if exact:
                assert K.bitwise_equal(sa, sb), f"call {ci} stream {s}: symbols differ (bitwise)"
            else:
                assert np.max(np.abs(sa - sb), initial=0) <= SYM_TOL


@pytest.mark.parametrize("sps,span", K.CONFIGS)
def test_single_call_bit_exact(sps, span):
    iq = K.batch_signals(5, seed0=10, sps=sps, span=span, n_bits=3000, snr_db=16)
    calls = [[iq.shape[1] // 2] * 5]
    assert_same(gpu_run(iq, calls, sps, span), oracle_run(iq, calls, sps, span))


@pytest.mark.parametrize("sps,span", K.CONFIGS)
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 6, 7])
def test_chunked_ragged_calls_bit_exact(sps, span, variant):
    """Every loop-kernel shape (qpsk_demod_params.loop_variant) on ragged calls,
    including 0/1/2/3-sample calls and calls longer than a round."""
    if variant == 3 and sps < 2:
        pytest.skip("16 x 128 needs sps >= 2 (the launcher never picks it below)")
    if variant in (4, 6, 7) and sps < 8:
        pytest.skip("24 x 128, 64 x 32 and 12 x 256 are sps >= 8 shapes (below it the launcher falls back to auto)")
    iq = K.batch_signals(4, seed0=20, sps=sps, span=span, n_bits=2400, snr_db=14)
    n = iq.shape[1] // 2
    rng = np.random.default_rng(sps)
    calls, left = [], np.full(4, n)
    sizes = [1, 2, 3, 0, 777, 5, 4096]
    k = 0
    while left.max() > 0:
        c = [int(min(left[s], sizes[(k + s) % len(sizes)] if k < 12 else rng.integers(100, 3000)))
             for s in range(4)]
        calls.append(c)
        left -= np.array(c)
        k += 1
    ref = oracle_run(iq, calls, sps, span)
    assert_same(gpu_run(iq, calls, sps, span, loop_variant=variant), ref)
    # the production bits-only kernel on the same ragged calls
    assert_same(gpu_run(iq, calls, sps, span, loop_variant=variant, want_syms=False), ref)


@pytest.mark.parametrize("variant", [4, 6, 7])
def test_long_round_shapes_many_streams_bit_exact(variant):
    """The 128- and 256-sample-round shapes over several workgroups (30
    streams: 2 x 15 rows of 24, or 3 x 10 rows of 12 with 22 shadow lanes each)
    with ragged per-stream call lengths, so streams end in different rounds."""
    sps, span, S = 8, 8, 30
    iq = K.batch_signals(S, seed0=77, sps=sps, span=span, n_bits=3000, snr_db=14)
    n = iq.shape[1] // 2
    rng = np.random.default_rng(variant)
    calls, used = [], np.zeros(S, np.int64)
    for _ in range(3):
        lens = rng.integers(0, n // 4, S)
        calls.append([int(v) for v in lens])
        used += lens
    calls.append([int(n - u) for u in used])
    ref = oracle_run(iq, calls, sps, span)
    assert_same(gpu_run(iq, calls, sps, span, loop_variant=variant), ref)
    assert_same(gpu_run(iq, calls, sps, span, loop_variant=variant, want_syms=False), ref)


@pytest.mark.parametrize("sps,span", [(30, 6), (100, 4), (200, 2), (300, 2), (1000, 1)])
def test_large_sps_multi_call_bit_exact(sps, span):
    """Samples per symbol up to 1000 (the reference's own testFullDemodChain
    runs sps 30), across calls shorter than one symbol too.  The queue the
    M&M keeps between calls is at most 3 samples whatever sps is
    (MuellerMuller.cs:123-133 drops min(baseIndex - 1, count - 3)); a symbol
    base past the end carries over as the state's base offset, not as
    samples."""
    iq = K.batch_signals(3, seed0=25, sps=sps, span=span, n_bits=300, snr_db=18)
    n = iq.shape[1] // 2
    calls, left, k = [], np.full(3, n), 0
    sizes = [1, 7, sps // 2, 3 * sps + 5, 0, 2 * sps - 1, 4096]
    while left.max() > 0:
        c = [int(min(left[s], sizes[(k + s) % len(sizes)])) for s in range(3)]
        calls.append(c)
        left -= np.array(c)
        k += 1
    assert_same(gpu_run(iq, calls, sps, span), oracle_run(iq, calls, sps, span))


def test_empty_call_keeps_state():
    iq = K.batch_signals(2, seed0=30, n_bits=1200)
    n = iq.shape[1] // 2
    calls = [[n // 2] * 2, [0, 0], [n - n // 2] * 2]
    assert_same(gpu_run(iq, calls, 8, 8), oracle_run(iq, calls, 8, 8))


def test_nondifferential_bit_exact():
    iq = K.batch_signals(3, seed0=40, sps=4, span=32, n_bits=2000, snr_db=20, differential=False)
    calls = [[iq.shape[1] // 2] * 3]
    assert_same(gpu_run(iq, calls, 4, 32, differential=False),
                oracle_run(iq, calls, 4, 32, differential=False))


def test_constellation_mode_shares_state():
    iq = K.batch_signals(3, seed0=50, n_bits=2000, snr_db=15)
    n = iq.shape[1] // 2
    calls = [[n // 3] * 3, [n // 3] * 3, [n - 2 * (n // 3)] * 3]
    modes = [Q.MODE_DEMODULATE, Q.MODE_CONSTELLATION, Q.MODE_DEMODULATE]
    assert_same(gpu_run(iq, calls, 8, 8, mode=modes), oracle_run(iq, calls, 8, 8, mode=modes))


@pytest.mark.parametrize("lanes", [4, 1, 16])
def test_other_vector_widths_bit_exact(lanes):
    iq = K.batch_signals(3, seed0=60, sps=8, span=8, n_bits=1500, snr_db=15)
    calls = [[5000] * 3, [iq.shape[1] // 2 - 5000] * 3]
    assert_same(gpu_run(iq, calls, 8, 8, vector_lanes=lanes), oracle_run(iq, calls, 8, 8, lanes=lanes))


def test_even_tap_count_generic_path():
    # sps 3, span 6 -> 19 taps (odd, generic); sps 3 span 5 -> 16 taps (even)
    for sps, span in [(3, 6), (3, 5)]:
        iq = K.batch_signals(2, seed0=70, sps=sps, span=span, n_bits=1500, snr_db=20)
        calls = [[iq.shape[1] // 2] * 2]
        assert_same(gpu_run(iq, calls, sps, span), oracle_run(iq, calls, sps, span))


def test_libm_oracle_bits_equal_symbols_close():
    iq = K.batch_signals(4, seed0=80, n_bits=4000, snr_db=14)
    calls = [[iq.shape[1] // 2] * 4]
    assert_same(gpu_run(iq, calls, 8, 8), oracle_run(iq, calls, 8, 8, trig=O.TRIG_LIBM), exact=False)


@pytest.mark.parametrize("lanes", [8, 4])
def test_fll_mode_bit_exact(lanes):
    """lanes 8: the systolic FLL kernel; other widths: the one-lane kernel."""
    iq = K.batch_signals(3, seed0=90, sps=8, span=8, n_bits=1200, cfo_hz=4000.0, snr_db=25)
    n = iq.shape[1] // 2
    calls = [[n // 2] * 3, [n - n // 2] * 3]
    assert_same(gpu_run(iq, calls, 8, 8, enable_fll=True, cfo_loop_bandwidth=1e-3, vector_lanes=lanes),
                oracle_run(iq, calls, 8, 8, enable_fll=True, cfo_loop_bw=1e-3, lanes=lanes))


def test_fll_ragged_chunks_bit_exact():
    """Systolic FLL (qpsk_fll.hip): ragged per-stream call lengths, calls shorter
    than one 8-sample block and than the 40-tap window, empty calls, and a
    batch that leaves most rows of the last workgroup empty."""
    S = 11
    iq = K.batch_signals(S, seed0=95, sps=8, span=8, n_bits=900, cfo_hz=-3000.0, snr_db=22)
    n = iq.shape[1] // 2
    rng = np.random.default_rng(7)
    calls, used = [], np.zeros(S, np.int64)
    for c in range(8):
        lens = rng.integers(0, 50, S) if c < 6 else np.full(S, 37)
        lens[c % S] = 0
        calls.append([int(v) for v in lens])
        used += lens
    calls.append([int(n - u) for u in used])
    assert_same(gpu_run(iq, calls, 8, 8, enable_fll=True, cfo_loop_bandwidth=1e-3),
                oracle_run(iq, calls, 8, 8, enable_fll=True, cfo_loop_bw=1e-3))


def test_state_checkpoint_roundtrip():
    iq = K.batch_signals(2, seed0=100, n_bits=1600, snr_db=15)
    n = iq.shape[1] // 2
    h = n // 2
    p = Q.params(K.FS, K.FS // 8, K.ALPHA, 8, max_samples_per_call=n)
    a = Q.BatchDemodulator(2, p)
    ba, na, _, _ = a.process(iq[:, : 2 * h])
    blob = a.get_state()
    b = Q.BatchDemodulator(2, p)
    b.set_state(blob)
    bb, nb, _, _ = b.process(iq[:, 2 * h:])
    ref = oracle_run(iq, [[h, h], [n - h, n - h]], 8, 8)
    for s in range(2):
        assert Q.unpack_bits(ba[s], int(na[s])) == ref[0][s][0]
        assert Q.unpack_bits(bb[s], int(nb[s])) == ref[1][s][0]
    # a blob is only accepted by a handle of its own shape and format
    hd = np.frombuffer(blob[: Q.STATE_HEADER_BYTES], dtype=np.uint32)
    assert hd[0] == 0x4B535051 and hd[1] == 2 and hd[2] == 2
    for bad in (blob[:-8], blob + b"\0" * 8, b"\0" * 4 + blob[4:], blob[:4] + b"\1\0\0\0" + blob[8:]):
        with pytest.raises(ValueError):   # QPSK_ERR_ARGUMENT
            b.set_state(bad)
    c = Q.BatchDemodulator(3, p)   # three streams: another layout
    with pytest.raises(ValueError):
        c.set_state(blob)
    c.close()
    a.close()
    b.close()


def test_mirror_test_at_data_level():
    """The reference's own procedure through the single-stream mirror class:
    same payload text as the oracle, frame for frame."""
    fs, rs, span = K.FS, K.FS // 8, 8
    g = Q.QPSKDeModulator(fs, rs, K.ALPHA, span, tsc=K.TSC)
    o = O.OracleDemod(fs, rs, K.ALPHA, span, tsc=K.TSC)
    tx = O.OracleNCO(100e6, fs, 1, 0, seed=11)
    rx = O.OracleNCO(100e6, fs, 1, 0, seed=22)
    ok = 0
    for _ in range(12):
        sig = O.modulate_text_utf8(fs, rs, K.PAYLOAD, "MESSAGE_START", "MESSAGE_STOP",
                                   rrc_alpha=K.ALPHA, rrc_span=span, tsc=K.TSC)
        sig = O.apply_lo_pair(tx, rx, sig)
        a = g.DeModulateTextUtf8(sig, "MESSAGE_START", "MESSAGE_STOP")
        b = o.DeModulateTextUtf8(sig, "MESSAGE_START", "MESSAGE_STOP")
        assert a == b
        ok += K.PAYLOAD in a
    assert ok >= 5


def test_mirror_errors():
    g = Q.QPSKDeModulator(K.FS, K.FS // 8, K.ALPHA, 8)
    with pytest.raises(ValueError):
        g.DeModulate(np.zeros(5, np.float32))
    assert g.DeModulate(np.zeros(0, np.float32)) == ""
    with pytest.raises(ValueError):
        g.DeModulateBytes(np.zeros(4, np.float32), b"", b"\x03")
    with pytest.raises(ValueError):
        Q.QPSKDeModulator(K.FS, K.FS // 8, 1.5, 8)


def test_synth_generated_batch_parity_and_ber():
    """GPU-generated clean batch: GPU bits == oracle bits on the same buffer, and
    most streams decode error-free after the symbol-sync pull-in.  (The
    reference's M&M loop is marginal on some start phases -- the oracle shows
    the same symbol slips -- so the BER bar is per-stream majority, not all.)"""
    S, n = 8, 1 << 16
    iq, tx = Q.synth_generate(S, n, K.FS, K.FS // 8, rrc_span=8, seed=123)
    host = iq.cpu().numpy()
    ref = oracle_run(host, [[n] * S], 8, 8)
    got = gpu_run(host, [[n] * S], 8, 8)
    assert_same(got, ref)
    txb = tx.cpu().numpy()
    clean = 0
    for s in range(S):
        rx = got[0][s][0]
        txs = Q.unpack_bits(txb[s], 2 * (n // 8))
        i = txs.find(rx[3000:3400])
        if i < 0:
            continue
        off = i - 3000
        m = min(len(rx), len(txs) - off) - 16
        a = np.frombuffer(rx[3000:m].encode(), np.uint8)
        r = np.frombuffer(txs[3000 + off:m + off].encode(), np.uint8)
        clean += int(np.count_nonzero(a != r) == 0)
    assert clean >= S // 2


def out_rows(S, ms, layout):
    """Device output rows.  "direct": word-aligned rows the loop kernel writes
    in place; "staged": a 1-byte-offset bit row of odd stride and an odd
    symbol stride, which take the staging buffers and the 2-D copies."""
    import torch
    if layout == "staged":
        bw = (2 * ms + 7) // 8 + 9
        bw += 1 - bw % 2
        bits = torch.zeros((S, bw + 1), dtype=torch.uint8, device="cuda")[:, 1:]
        sy = torch.zeros((S, 2 * ms + 1), dtype=torch.float32, device="cuda")
    else:
        bits = torch.zeros((S, ((2 * ms + 7) // 8 + 63) // 64 * 64), dtype=torch.uint8, device="cuda")
        sy = torch.zeros((S, 2 * ms), dtype=torch.float32, device="cuda")
    return bits, sy


def async_run(iq2d, calls, sps, span, sync_every=0, layout=None, **kw):
    """The same call sequence through qpsk_demod_process_async (front stage of
    call k+1 overlapping the back stage of call k), every call's outputs in
    their own device rows, one pipeline_wait at the end.  sync_every > 0 makes
    every sync_every-th call a synchronous process() (mixed ordering).
    layout: None (rows as a caller would size them), or out_rows' layouts."""
    import torch
    S = iq2d.shape[0]
    nmax = max(max(c) for c in calls)
    p = Q.params(K.FS, K.FS // sps, K.ALPHA, span, max_samples_per_call=nmax + 8, **kw)
    b = Q.BatchDemodulator(S, p)
    stream = torch.cuda.Stream()
    b.set_stream(stream.cuda_stream)
    ms = max(b.max_symbols(nmax), 1)
    pos = np.zeros(S, dtype=np.int64)
    outs = []
    with torch.cuda.stream(stream):
        for ci, lens in enumerate(calls):
            n = int(max(lens))
            x = np.zeros((S, 2 * max(n, 1)), np.float32)
            for s in range(S):
                x[s, : 2 * lens[s]] = iq2d[s, 2 * pos[s]: 2 * (pos[s] + lens[s])]
            xd = torch.from_numpy(x).to("cuda", non_blocking=False)
            if layout:
                bits, sy = out_rows(S, ms, layout)
            else:
                bits = torch.zeros((S, (2 * ms + 7) // 8 + 8), dtype=torch.uint8, device="cuda")
                sy = torch.zeros((S, 2 * ms), dtype=torch.float32, device="cuda")
            nb = torch.zeros(S, dtype=torch.int64, device="cuda")
            ns = torch.zeros(S, dtype=torch.int64, device="cuda")
            uniform = all(l == lens[0] for l in lens)
            if sync_every and ci % sync_every == sync_every - 1:
                assert uniform
                b.process_device(xd, n, bits, nb, syms_dev=sy, n_syms_dev=ns)
            else:
                b.process_device_async(xd, n, bits, nb, syms_dev=sy, n_syms_dev=ns,
                                       lengths=None if uniform else np.array(lens))
            outs.append((xd, bits, nb, sy, ns))
            pos += np.array(lens)
    depth = b.pipeline_depth()
    b.pipeline_wait()
    torch.cuda.synchronize()
    res = []
    for _, bits, nb, sy, ns in outs:
        bits, nb, sy, ns = bits.cpu().numpy(), nb.cpu().numpy(), sy.cpu().numpy(), ns.cpu().numpy()
        res.append([(Q.unpack_bits(bits[s], int(nb[s])), sy[s, : 2 * int(ns[s])].copy()) for s in range(S)])
    b.close()
    return res, depth


@pytest.mark.parametrize("layout", ["direct", "staged"])
@pytest.mark.parametrize("sync_every,fll", [(0, False), (2, False), (0, True)])
def test_device_output_rows_in_place_or_staged(layout, sync_every, fll):
    """Device calls whose rows the loop kernel can address are written in
    place (no 2-D copy behind it); misaligned or odd-stride rows go through
    the staging buffers.  Both, synchronous and pipelined (with the FLL: the
    loop kernel issued by the next call), equal the oracle."""
    kw = dict(enable_fll=True, cfo_loop_bandwidth=1e-3) if fll else {}
    okw = dict(enable_fll=True, cfo_loop_bw=1e-3) if fll else {}
    iq = K.batch_signals(4, seed0=470, sps=8, span=8, n_bits=2400, snr_db=16, cfo_hz=2000.0 if fll else 0.0)
    n = iq.shape[1] // 2
    calls = [[n // 4] * 4, [n // 3] * 4, [n // 5] * 4, [n - n // 4 - n // 3 - n // 5] * 4]
    got, _ = async_run(iq, calls, 8, 8, sync_every=sync_every, layout=layout, **kw)
    assert_same(got, oracle_run(iq, calls, 8, 8, **okw))


@pytest.mark.parametrize("fll", [False, True])
def test_pipelined_calls_bit_exact(fll):
    """qpsk_demod_process_async: uniform and ragged calls, empty calls, with and
    without the FLL (whose front stage is the FLL instead of the FIR)."""
    kw = dict(enable_fll=True, cfo_loop_bandwidth=1e-3) if fll else {}
    okw = dict(enable_fll=True, cfo_loop_bw=1e-3) if fll else {}
    iq = K.batch_signals(5, seed0=400, sps=8, span=8, n_bits=2400, snr_db=16,
                         cfo_hz=3000.0 if fll else 0.0)
    n = iq.shape[1] // 2
    rng = np.random.default_rng(11)
    calls, used = [], np.zeros(5, np.int64)
    for c in range(7):
        lens = np.full(5, 1500) if c % 3 == 0 else rng.integers(0, 2500, 5)
        if c == 4:
            lens[:] = 0
        calls.append([int(v) for v in lens])
        used += lens
    calls.append([int(n - u) for u in used])
    got, depth = async_run(iq, calls, 8, 8, **kw)
    assert depth == 2
    assert_same(got, oracle_run(iq, calls, 8, 8, **okw))


def test_pipelined_mixed_with_sync_calls():
    """Synchronous process() calls interleaved with pipelined ones keep one order."""
    iq = K.batch_signals(3, seed0=410, sps=4, span=32, n_bits=3000, snr_db=16)
    n = iq.shape[1] // 2
    k = n // 6
    calls = [[k] * 3 for _ in range(5)] + [[n - 5 * k] * 3]
    got, _ = async_run(iq, calls, 4, 32, sync_every=2)
    assert_same(got, oracle_run(iq, calls, 4, 32))


def test_huge_amplitude_takes_the_costas_rollback_path():
    """Samples scaled by 1e12 drive theta far past the table reduction's range
    (|theta| > 1e6): the loop kernel's fast pass detects it and redoes the round
    with the full-range sincos, matching the oracle bit for bit."""
    iq = K.batch_signals(3, seed0=300, sps=8, span=8, n_bits=800, snr_db=20) * np.float32(1e12)
    n = iq.shape[1] // 2
    calls = [[n // 3] * 3, [n - n // 3] * 3]
    got, ref = gpu_run(iq, calls, 8, 8), oracle_run(iq, calls, 8, 8)
    for ci, (ra, rb) in enumerate(zip(got, ref)):
        for s, ((ba, sa), (bb, sb)) in enumerate(zip(ra, rb)):
            assert ba == bb, f"call {ci} stream {s}: bits differ"
            assert K.bitwise_equal(sa, sb), f"call {ci} stream {s}"
    # (with |pe| ~ 1e12 the first symbol already moves freq by cb*pe ~ 1e10, so
    # theta leaves [-1e6, 1e6] within a round)


@pytest.mark.parametrize("sps,span", [(8, 8), (4, 32)])
def test_degenerate_streams_bit_exact(sps, span):
    """Streams the synthetic batches never hold, beside normal ones, against
    the oracle bit for bit: all zeros (every decision at +0, the TED and phase
    error exactly 0), a signal scaled into the subnormal range (products and
    interpolations below 2^-126: the kernels must not flush them), a constant
    DC level, and a signal with a zeroed gap spanning calls."""
    iq = K.batch_signals(6, seed0=700, sps=sps, span=span, n_bits=1200, snr_db=18)
    iq[1] = 0.0
    iq[2] = iq[2] * np.float32(1e-39)
    assert np.count_nonzero(np.abs(iq[2]) < np.float32(2.0 ** -126)) > iq.shape[1] // 2
    iq[3] = np.float32(0.25)
    n = iq.shape[1] // 2
    iq[4, 2 * (n // 3): 2 * (n // 3 + 700)] = 0.0
    calls = [[n // 3 + 100] * 6, [0, 5, 17, 1, 300, 2], [n - n // 3 - 100, n - n // 3 - 105,
                                                        n - n // 3 - 117, n - n // 3 - 101,
                                                        n - n // 3 - 400, n - n // 3 - 102]]
    got, ref = gpu_run(iq, calls, sps, span), oracle_run(iq, calls, sps, span)
    for ci, (ra, rb) in enumerate(zip(got, ref)):
        for s, ((ba, sa), (bb, sb)) in enumerate(zip(ra, rb)):
            assert ba == bb, f"call {ci} stream {s}: bits differ"
            assert K.bitwise_equal(sa, sb), f"call {ci} stream {s}: symbols"


def ring_run(iq2d, calls, sps, span, depth=2, zero_copy=False, **kw):
    """The host-fed ring (qpsk_rx_*): submit every call, collecting only when the
    ring is full, so uploads and computes of consecutive calls overlap."""
    S = iq2d.shape[0]
    p = Q.params(K.FS, K.FS // sps, K.ALPHA, span, max_samples_per_call=max(max(c) for c in calls) + 8, **kw)
    b = Q.BatchDemodulator(S, p)
    ring = Q.HostRing(b, depth)
    pos = np.zeros(S, dtype=np.int64)
    out, pending = [], 0

    def collect():
        bits, nb, _ = ring.collect()
        out.append([(Q.unpack_bits(bits[s], int(nb[s])), None) for s in range(S)])

    for lens in calls:
        n = int(max(lens))
        uniform = all(l == lens[0] for l in lens)
        if pending == depth:
            collect()
            pending -= 1
        if zero_copy:
            slot = ring.next_slot()
            for s in range(S):
                slot[s, : 2 * lens[s]] = iq2d[s, 2 * pos[s]: 2 * (pos[s] + lens[s])]
            ring.submit(None, n, None if uniform else np.array(lens))
        else:
            x = np.zeros((S, 2 * max(n, 1)), np.float32)
            for s in range(S):
                x[s, : 2 * lens[s]] = iq2d[s, 2 * pos[s]: 2 * (pos[s] + lens[s])]
            ring.submit(x, n, None if uniform else np.array(lens))
        pending += 1
        pos += np.array(lens)
    while pending:
        collect()
        pending -= 1
    ring.close()
    b.close()
    return out


def assert_same_bits(got, want):
    for ci, (ra, rb) in enumerate(zip(got, want)):
        for s, ((ba, _), (bb, _)) in enumerate(zip(ra, rb)):
            assert ba == bb, f"call {ci} stream {s}: bits differ ({len(ba)} vs {len(bb)})"


@pytest.mark.parametrize("depth,zero_copy,fll", [(2, False, False), (3, True, False), (2, True, True)])
def test_host_ring_bit_exact(depth, zero_copy, fll):
    """The streaming front-end (ModDemodOverSDR.cs:116-183 receive loop): uniform,
    ragged and empty chunks through the pinned ring give the oracle's bits."""
    kw = dict(enable_fll=True, cfo_loop_bandwidth=1e-3) if fll else {}
    okw = dict(enable_fll=True, cfo_loop_bw=1e-3) if fll else {}
    iq = K.batch_signals(4, seed0=500 + depth, sps=8, span=8, n_bits=2400, snr_db=16,
                         cfo_hz=3000.0 if fll else 0.0)
    n = iq.shape[1] // 2
    rng = np.random.default_rng(21 + depth)
    calls, used = [], np.zeros(4, np.int64)
    for c in range(7):
        lens = np.full(4, 1300) if c % 3 == 0 else rng.integers(0, 2200, 4)
        if c == 5:
            lens[:] = 0
        calls.append([int(v) for v in lens])
        used += lens
    calls.append([int(n - u) for u in used])
    got = ring_run(iq, calls, 8, 8, depth=depth, zero_copy=zero_copy, **kw)
    assert_same_bits(got, oracle_run(iq, calls, 8, 8, **okw))


def test_host_ring_errors():
    p = Q.params(K.FS, K.FS // 8, K.ALPHA, 8, max_samples_per_call=4096)
    b = Q.BatchDemodulator(2, p)
    with pytest.raises(ValueError):
        Q.HostRing(b, 1)
    ring = Q.HostRing(b, 2)
    with pytest.raises(Q.QPSKError):
        ring.collect()                    # nothing outstanding
    x = np.zeros((2, 2 * 1000), np.float32)
    ring.submit(x, 1000)
    ring.submit(x, 1000)
    with pytest.raises(Q.QPSKError):
        ring.submit(x, 1000)              # both slots hold uncollected chunks
    ring.collect()
    with pytest.raises(ValueError):
        ring.submit(np.zeros((2, 2 * 5000), np.float32), 5000)   # > max_samples_per_call
    ring.collect()
    ring.close()
    b.close()


def test_c_abi_demo_from_plain_c():
    """The boundary from plain C, the way a cgo / JNI / P/Invoke binding (or a
    C++ multi-GPU driver) calls it: tools/c_abi_demo (built by build())
    demodulates ragged calls through qpsk_demod_process, the qpsk_rx ring and a
    two-shard qpsk_demod_group on device 0, and checks every call's bits
    against the oracle's DeModulate."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tools", "bin", "c_abi_demo")
    assert os.path.exists(exe), "run __graft_entry__.build() (make -f tools/c_abi_demo.mk)"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bits identical to the oracle" in r.stdout and "2-shard group" in r.stdout


@pytest.mark.parametrize("layout", ["direct", "staged"])
@pytest.mark.parametrize("pipelined", [False, True])
def test_device_constellation_rows_in_place_or_staged(layout, pipelined):
    """deModulateConstellation (QPSKDeModulator.cs:427-455) on device rows:
    symbols written in place or through the staging copy, interleaved with
    DeModulate calls on the same state, synchronous and pipelined."""
    import torch
    S = 4
    iq = K.batch_signals(S, seed0=480, sps=8, span=8, n_bits=2400, snr_db=16)
    n = iq.shape[1] // 2
    calls = [[n // 3] * S, [n // 3] * S, [n - 2 * (n // 3)] * S]
    modes = [Q.MODE_CONSTELLATION, Q.MODE_DEMODULATE, Q.MODE_CONSTELLATION]
    b = Q.BatchDemodulator(S, Q.params(K.FS, K.FS // 8, K.ALPHA, 8, max_samples_per_call=n))
    stream = torch.cuda.Stream()
    b.set_stream(stream.cuda_stream)
    ms = b.max_symbols(n)
    outs, pos = [], 0
    with torch.cuda.stream(stream):
        for lens, m in zip(calls, modes):
            k = lens[0]
            xd = torch.from_numpy(np.ascontiguousarray(iq[:, 2 * pos: 2 * (pos + k)])).to("cuda")
            bits, sy = out_rows(S, ms, layout)
            nb = torch.zeros(S, dtype=torch.int64, device="cuda")
            ns = torch.zeros(S, dtype=torch.int64, device="cuda")
            f = b.process_device_async if pipelined else b.process_device
            f(xd, k, bits if m == Q.MODE_DEMODULATE else None, nb if m == Q.MODE_DEMODULATE else None,
              mode=m, syms_dev=sy, n_syms_dev=ns)
            outs.append((xd, bits, nb, sy, ns, m))
            pos += k
    b.pipeline_wait()
    torch.cuda.synchronize()
    got = []
    for _, bits, nb, sy, ns, m in outs:
        bits, nb, sy, ns = bits.cpu().numpy(), nb.cpu().numpy(), sy.cpu().numpy(), ns.cpu().numpy()
        got.append([(Q.unpack_bits(bits[s], int(nb[s])) if m == Q.MODE_DEMODULATE else "",
                     sy[s, : 2 * int(ns[s])].copy()) for s in range(S)])
    b.close()
    assert_same(got, oracle_run(iq, calls, 8, 8, mode=modes))
