"""GPU parity, round 2: scale, libm trig in FLL mode, chunked calls, non-finite
samples, status flags, the GPU modulator and synthesiser against the oracle.

Every test goes through the C ABI (qpsk_amd) and compares with the CPU oracle
(oracle/) on the same inputs.
"""
import numpy as np
import pytest

import common as K
import oracle as O
import qpsk_amd as Q
from test_gpu_parity import SYM_TOL, assert_same, gpu_run, oracle_run

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need an MI355X")
    yield


def _rows(t, idx):
    return np.concatenate([t[i: i + 1].cpu().numpy() for i in idx])


def test_rows_past_4gib_bit_exact():
    """640 streams x 2^20 samples: the last rows start ~5 GiB into the input and
    MF buffers.  Their bits AND symbols equal the oracle's (portable trig),
    as do the first row's."""
    import torch
    S, n = 640, 1 << 20
    iq, _ = Q.synth_generate(S, n, K.FS, K.FS // 8, rrc_span=8, seed=777)
    assert iq.stride(0) * 4 * (S - 1) > (4 << 30)
    b = Q.BatchDemodulator(S, Q.params(K.FS, K.FS // 8, K.ALPHA, 8, max_samples_per_call=n))
    ms = b.max_symbols(n)
    dev = iq.device
    bits = torch.zeros((S, (2 * ms + 7) // 8 + 8), dtype=torch.uint8, device=dev)
    nb = torch.zeros(S, dtype=torch.int64, device=dev)
    syms = torch.zeros((S, 2 * ms), dtype=torch.float32, device=dev)
    ns = torch.zeros(S, dtype=torch.int64, device=dev)
    b.process_device(iq, n, bits, nb, syms_dev=syms, n_syms_dev=ns)
    torch.cuda.synchronize()
    idx = [0, S - 2, S - 1]
    host = _rows(iq, idx)
    gb, gnb, gs, gns = _rows(bits, idx), _rows(nb, idx), _rows(syms, idx), _rows(ns, idx)
    for i, s in enumerate(idx):
        ob, osy, _ = K.oracle_for(8, 8).demodulate_ex(host[i])
        assert Q.unpack_bits(gb[i], int(gnb[i])) == ob, f"stream {s}: bits"
        assert K.bitwise_equal(gs[i, : 2 * int(gns[i])], osy), f"stream {s}: symbols"
    assert b.status() == 0
    b.close()


@pytest.mark.parametrize("seed", [500, 510])
def test_fll_mode_vs_libm_oracle(seed):
    """FLL on, against the oracle calling the real glibc (MathF.Sin/Cos and
    Math.Sin/Cos of .NET on Linux): the FLL's float trig is glibc's own
    algorithm (qpsk_sincosf.h), so bits are identical; the Costas double trig
    is the portable table, so symbols agree within SYM_TOL."""
    iq = K.batch_signals(4, seed0=seed, sps=8, span=8, n_bits=6000, cfo_hz=4500.0, multipath=True,
                         snr_db=20)
    n = iq.shape[1] // 2
    calls = [[n // 3] * 4, [n - n // 3] * 4]
    got = gpu_run(iq, calls, 8, 8, enable_fll=True, cfo_loop_bandwidth=1e-3)
    ref = oracle_run(iq, calls, 8, 8, enable_fll=True, cfo_loop_bw=1e-3, trig=O.TRIG_LIBM)
    assert_same(got, ref, exact=False)


def test_fll_mode_default_bandwidth_vs_libm_oracle():
    """The C5 FLL settings (CFOLoopBandwith default) on a longer impaired stream."""
    iq = K.batch_signals(2, seed0=530, sps=8, span=8, n_bits=20000, cfo_hz=5000.0, multipath=True,
                         snr_db=20)
    calls = [[iq.shape[1] // 2] * 2]
    got = gpu_run(iq, calls, 8, 8, enable_fll=True)
    ref = oracle_run(iq, calls, 8, 8, enable_fll=True, trig=O.TRIG_LIBM)
    assert_same(got, ref, exact=False)


@pytest.mark.parametrize("ragged", [False, True])
def test_call_longer_than_capacity_is_chunked(ragged):
    """QPSKDeModulator.DeModulate takes any span (QPSKDeModulator.cs:345-360): a
    call 3x max_samples_per_call runs as internal chunks and returns exactly
    one oracle DeModulate call's bits and symbols (host memory)."""
    S = 3
    iq = K.batch_signals(S, seed0=600, sps=8, span=8, n_bits=3000, snr_db=18)
    n = iq.shape[1] // 2
    cap = n // 3 - 5
    lens = np.array([n, n - 777, n - 2 * cap - 3]) if ragged else None
    b = Q.BatchDemodulator(S, Q.params(K.FS, K.FS // 8, K.ALPHA, 8, max_samples_per_call=cap))
    bits, nb, syms, ns = b.process(iq, lengths=lens, want_syms=True)
    for s in range(S):
        m = int(lens[s]) if ragged else n
        ob, osy, _ = K.oracle_for(8, 8).demodulate_ex(iq[s, : 2 * m])
        assert Q.unpack_bits(bits[s], int(nb[s])) == ob, f"stream {s}: bits"
        assert K.bitwise_equal(syms[s, : 2 * int(ns[s])], osy), f"stream {s}: symbols"
    b.close()


def test_chunked_device_and_pipelined_calls():
    """The same oversized call on device memory, synchronous and pipelined,
    twice in a row (state carries across the chunked calls)."""
    import torch
    S = 2
    iq = K.batch_signals(S, seed0=620, sps=8, span=8, n_bits=2400, snr_db=18)
    n = iq.shape[1] // 2
    half = n // 2
    cap = half // 2 - 7
    ref = oracle_run(iq, [[half] * S, [n - half] * S], 8, 8)
    for pipelined in (False, True):
        b = Q.BatchDemodulator(S, Q.params(K.FS, K.FS // 8, K.ALPHA, 8, max_samples_per_call=cap))
        ms = b.max_symbols(n)
        x = torch.from_numpy(iq).cuda()
        for ci, (lo, hi) in enumerate([(0, half), (half, n)]):
            xc = x[:, 2 * lo: 2 * hi].contiguous()
            bits = torch.zeros((S, (2 * ms + 7) // 8 + 8), dtype=torch.uint8, device=x.device)
            nb = torch.zeros(S, dtype=torch.int64, device=x.device)
            sy = torch.zeros((S, 2 * ms), dtype=torch.float32, device=x.device)
            ns = torch.zeros(S, dtype=torch.int64, device=x.device)
            if pipelined:
                b.process_device_async(xc, hi - lo, bits, nb, syms_dev=sy, n_syms_dev=ns)
                b.pipeline_wait()
            else:
                b.process_device(xc, hi - lo, bits, nb, syms_dev=sy, n_syms_dev=ns)
            torch.cuda.synchronize()
            for s in range(S):
                rb, rs = ref[ci][s]
                assert Q.unpack_bits(bits[s].cpu().numpy(), int(nb[s])) == rb, (pipelined, ci, s)
                assert K.bitwise_equal(sy[s, : 2 * int(ns[s])].cpu().numpy(), rs), (pipelined, ci, s)
        b.close()


def test_nonfinite_samples_in_the_matched_filter():
    """NaN in I of one stream, +Inf in Q of another, -Inf in both of a third:
    the reference's full complex products ((hI*xI) - (hQ*xQ) with hQ = +0,
    FIRFilter.cs:172-173) turn 0*Inf into NaN in the other component too.  The
    GPU matched filter equals the oracle's, NaN for NaN (payload aside); the
    finite stream is untouched, and the timing loop reports the stall
    (QPSK_STATUS_NONFINITE_TIMING)."""
    S = 4
    iq = K.batch_signals(S, seed0=640, sps=8, span=8, n_bits=1500, snr_db=18)
    iq[1, 2 * 1000] = np.nan
    iq[2, 2 * 2000 + 1] = np.inf
    iq[3, 2 * 3000] = -np.inf
    iq[3, 2 * 3000 + 1] = -np.inf
    n = iq.shape[1] // 2
    b = Q.BatchDemodulator(S, Q.params(K.FS, K.FS // 8, K.ALPHA, 8, max_samples_per_call=n))
    with pytest.raises(Q.QPSKError, match="non-finite"):
        b.process(iq)
    mf = b.last_mf(n)
    taps = b.rrc_taps()
    taps_iq = np.zeros(2 * taps.size, np.float32)
    taps_iq[0::2] = taps
    for s in range(S):
        ref = O.oracle_fir(taps_iq, iq[s])
        assert K.bitwise_equal(mf[s], ref, nan_any_payload=True), f"stream {s}"
        if s > 0:
            assert np.isnan(mf[s]).any()
    assert b.status() & Q.STATUS_NONFINITE_TIMING
    assert b.status() == 0          # cleared by the read
    b.close()


def test_nonfinite_leaves_other_streams_bit_exact():
    import torch
    S = 3
    iq = K.batch_signals(S, seed0=660, sps=8, span=8, n_bits=1500, snr_db=18)
    iq[1, 2 * 500 + 1] = np.nan
    n = iq.shape[1] // 2
    b = Q.BatchDemodulator(S, Q.params(K.FS, K.FS // 8, K.ALPHA, 8, max_samples_per_call=n))
    x = torch.from_numpy(iq).cuda()
    ms = b.max_symbols(n)
    bits = torch.zeros((S, (2 * ms + 7) // 8 + 8), dtype=torch.uint8, device=x.device)
    nb = torch.zeros(S, dtype=torch.int64, device=x.device)
    b.process_device(x, n, bits, nb)
    assert b.status() == Q.STATUS_NONFINITE_TIMING
    for s in (0, 2):
        ob, _, _ = K.oracle_for(8, 8).demodulate_ex(iq[s])
        assert Q.unpack_bits(bits[s].cpu().numpy(), int(nb[s])) == ob
    b.close()


def test_oracle_follows_dotnet_nan_timing():
    """The oracle restates .NET 9: (int)Math.Floor(NaN) = 0 pins baseIndex at 0
    and CubicLagrange4 reads _bufIQ[-2] on a fresh buffer: IndexOutOfRange."""
    iq = K.batch_signals(1, seed0=680, sps=8, span=8, n_bits=400, snr_db=18)[0].copy()
    iq[2 * 50] = np.nan
    with pytest.raises(IndexError):
        K.oracle_for(8, 8).DeModulate(iq)


def test_synth_clean_matches_oracle_modulate():
    """qpsk_synth_generate with no carrier (lo_ppm = cfo_hz = 0) is
    QPSKModulator.Modulate (QPSKModulator.cs:104-167) of its own payload bits:
    equal to the oracle's modulate within 1e-6 (the synthesiser keeps
    1/sqrt2 in double where the modulator rounds it to float)."""
    for sps, span in ((8, 8), (4, 32)):
        S, n = 3, 20000
        iq, tx = Q.synth_generate(S, n, K.FS, K.FS // sps, rrc_span=span, seed=4242, lo_ppm=0.0)
        got = iq.cpu().numpy()
        txb = tx.cpu().numpy()
        T = span * sps + 1
        nsym = (n + (T - 1) // 2) // sps + 2
        for s in range(S):
            bits = Q.unpack_bits(txb[s], 2 * nsym)
            ref = O.modulate(K.FS, K.FS // sps, bits, rrc_alpha=K.ALPHA, rrc_span=span)
            assert ref.size >= 2 * n
            assert np.max(np.abs(got[s] - ref[: 2 * n])) <= 1e-6, (sps, s)


@pytest.mark.parametrize("diff,tsc,pulse", [(True, None, True), (True, K.TSC, True), (False, None, True),
                                            (True, K.TSC, False), (False, "0110", False)])
def test_gpu_modulator_bit_exact_vs_oracle(diff, tsc, pulse):
    """QPSKModulator on the GPU vs the oracle's restatement (direct double
    convolution of fftFilter): bit-identical float output, odd lengths too."""
    rng = np.random.default_rng(7)
    for sps, span, alpha in ((8, 8, 0.4), (2, 10, 0.9), (4, 32, 0.35)):
        m = Q.QPSKModulator(K.FS, K.FS // sps, alpha, span, differentialEncoding=diff, tsc=tsc)
        for nbits in (0, 1, 2, 7, 1001, 4000):
            data = K.random_bits(rng, nbits)
            got = m.Modulate(data, pulse)
            ref = O.modulate(K.FS, K.FS // sps, data, rrc_alpha=alpha, rrc_span=span, differential=diff,
                             tsc=tsc, pulse_shaping=pulse)
            assert got.shape == ref.shape, (sps, nbits)
            assert np.array_equal(got, ref), (sps, nbits)
        m.close()


def test_gpu_modulator_batch_bytes_and_text():
    m = Q.QPSKModulator(K.FS, K.FS // 8, K.ALPHA, 8)
    got = m.ModulateTextUtf8("The Quick Brown fox jump yes yes man good!")
    ref = O.modulate_text_utf8(K.FS, K.FS // 8, "The Quick Brown fox jump yes yes man good!",
                               rrc_alpha=K.ALPHA, rrc_span=8)
    assert np.array_equal(got, ref)
    got = m.ModulateBytes(b"\x00\xffpayload", b"START", b"STOP")
    ref = O.modulate_bytes(K.FS, K.FS // 8, b"\x00\xffpayload", b"START", b"STOP", rrc_alpha=K.ALPHA,
                           rrc_span=8)
    assert np.array_equal(got, ref)
    with pytest.raises(ValueError):
        m.ModulateBytes(b"x", b"", b"STOP")
    # batched: ragged rows in one call
    rng = np.random.default_rng(11)
    strs = [K.random_bits(rng, k) for k in (10, 333, 2000, 0)]
    rows = np.zeros((4, 256), np.uint8)
    for i, st in enumerate(strs):
        if st:
            p = Q.pack_bits(st)
            rows[i, : p.size] = p
    outs = m.modulate_batch(rows, [len(x) for x in strs])
    for st, o in zip(strs, outs):
        assert np.array_equal(o, O.modulate(K.FS, K.FS // 8, st, rrc_alpha=K.ALPHA, rrc_span=8))
    m.close()


def test_modulate_then_demodulate_round_trip():
    """TX on the GPU -> RX on the GPU: testAtDataLevel's frames come back."""
    m = Q.QPSKModulator(K.FS, K.FS // 8, K.ALPHA, 8, tsc=K.TSC)
    d = Q.QPSKDeModulator(K.FS, K.FS // 8, K.ALPHA, 8, tsc=K.TSC)
    texts = []
    for k in range(6):
        sig = m.ModulateTextUtf8(f"frame {k}: " + K.PAYLOAD)
        texts.append(d.DeModulateTextUtf8(sig))
    assert sum(t.endswith(K.PAYLOAD) for t in texts) >= 3


@pytest.mark.parametrize("fll", [False, True])
def test_iq_balance_prestage_bit_exact(fll):
    """The optional IQ_Balancer pre-stage (IQ Balancer.cs:15-25) on a signal
    with a DC offset, in ragged chunked calls, sync and pipelined: bits and
    symbols equal the oracle with the same pre-stage."""
    S = 3
    iq = K.batch_signals(S, seed0=700, sps=8, span=8, n_bits=2000, snr_db=18)
    iq[:, 0::2] += 0.3
    iq[:, 1::2] -= 0.2
    n = iq.shape[1] // 2
    calls = [[n // 3, n // 2, 100], [n - n // 3, n - n // 2, n - 100]]
    kw = dict(enable_fll=fll, cfo_loop_bandwidth=1e-3) if fll else {}
    okw = dict(enable_fll=fll, cfo_loop_bw=1e-3) if fll else {}
    got = gpu_run(iq, calls, 8, 8, iq_balance=True, **kw)
    ref = oracle_run(iq, calls, 8, 8, iq_balance=True, **okw)
    assert_same(got, ref)
    from test_gpu_parity import async_run
    got_async, _ = async_run(iq, calls, 8, 8, iq_balance=True, **kw)
    assert_same(got_async, ref)


def test_chunked_host_call_reports_nonfinite():
    """A host-memory call longer than max_samples_per_call runs as internal
    chunks; a NaN reaching the timing loop in any chunk fails the call with
    the same error as an unchunked call (QPSK_ERR_STATE, 'non-finite'), and the
    handle's status keeps the flag until read."""
    S = 2
    iq = K.batch_signals(S, seed0=690, sps=8, span=8, n_bits=1500, snr_db=18)
    n = iq.shape[1] // 2
    cap = n // 3
    iq[1, 2 * (cap + 100)] = np.nan          # inside the second chunk
    b = Q.BatchDemodulator(S, Q.params(K.FS, K.FS // 8, K.ALPHA, 8, max_samples_per_call=cap))
    with pytest.raises(Q.QPSKError, match="non-finite"):
        b.process(iq)
    assert b.status() & Q.STATUS_NONFINITE_TIMING
    assert b.status() == 0
    # a clean call afterwards on a fresh handle state succeeds and matches the oracle
    b.close()
    clean = K.batch_signals(S, seed0=691, sps=8, span=8, n_bits=1500, snr_db=18)
    b = Q.BatchDemodulator(S, Q.params(K.FS, K.FS // 8, K.ALPHA, 8, max_samples_per_call=cap))
    bits, nb, _, _ = b.process(clean)
    for s in range(S):
        assert Q.unpack_bits(bits[s], int(nb[s])) == K.oracle_for(8, 8).DeModulate(clean[s])
    b.close()


@pytest.mark.parametrize("fll", [False, True])
def test_launch_times_and_kernel_clocks(fll):
    """enable_timing: every timed call records its kernels' own spans and
    clock samples (qpsk_demod_launch_times / kernel_clocks), pipelined calls
    included; the FLL column is empty with the FLL off; enable_timing restarts
    the record; results do not change with timing on."""
    import torch
    S, n = 64, 1 << 15
    iq = torch.from_numpy(K.batch_signals(S, seed0=1300, sps=8, span=8, n_bits=2 * n // 8 + 64,
                                          snr_db=18)[:, : 2 * n].copy()).cuda()
    kw = dict(enable_fll=True, cfo_loop_bandwidth=1e-3) if fll else {}
    b = Q.BatchDemodulator(S, Q.params(K.FS, K.FS // 8, K.ALPHA, 8, max_samples_per_call=n, **kw))
    ms = b.max_symbols(n)
    bits = torch.zeros((S, ((2 * ms + 7) // 8 + 63) // 64 * 64), dtype=torch.uint8, device="cuda")
    nb = torch.zeros(S, dtype=torch.int64, device="cuda")
    b.process_device_async(iq, n, bits, nb)      # untimed
    b.enable_timing(True)
    for _ in range(3):
        b.process_device_async(iq, n, bits, nb)
    b.pipeline_wait()
    lt, kc, st = b.launch_times(), b.kernel_clocks(), b.stage_times()
    assert lt.shape == (3, 4) and kc.shape == (3, 3)
    assert (lt[:, 1] > 0).all() and (lt[:, 2] > 0).all()
    assert ((lt[:, 0] > 0) == fll).all()
    assert (lt[:, 3] >= lt[:, :3].max(axis=1) * 0.999).all()
    for j, ran in ((0, fll), (1, True), (2, True)):
        if ran:
            assert ((kc[:, j] > 0.3) & (kc[:, j] < 3.5)).all(), kc
        else:
            assert (kc[:, j] == 0).all()
    assert abs(st["fir"] - lt[:, 1].mean()) < 1e-3 and abs(st["loop"] - lt[:, 2].mean()) < 1e-3
    b.enable_timing(True)
    assert b.launch_times().shape == (0, 4)
    b.process_device_async(iq, n, bits, nb)
    b.pipeline_wait()
    assert b.launch_times().shape == (1, 4)
    b.enable_timing(False)
    b.close()
