"""Framer and TSC search: the host framer and the device-resident framer
(include/qpsk_demod.h, qpsk_framer_dev.hip) against the string-level
restatement of DeModulateBytes (refmodel.RefFramer, QPSKDeModulator.cs:169-259)
and str.find (the TSC strip, :413-422).

The call sequences are built to hit every branch of the reference state
machine: markers straddling call boundaries (the carry tail, :233-235), all 8
lock offsets, frames that open and close in one call, frames spanning many
calls, end markers straddling calls, calls whose TSC search failed (rxBits
empty, :179-180), empty calls, ring overflow with resync (:215-220, :241-245),
and a marker change between calls (markers are per-call arguments).
"""
import numpy as np
import pytest

import common as K
import oracle as O
import qpsk_amd as Q
from refmodel import RefFramer


def rand_bytes(rng, n):
    return bytes(rng.integers(0, 256, n, dtype=np.uint8))


def to_bits(b: bytes) -> str:
    return "".join(format(v, "08b") for v in b)


def make_stream(rng, start, end, n_frames, noise_bits=(0, 300), payload=(0, 40)):
    """Noise, then frames (start, payload bytes, end) at arbitrary bit offsets."""
    out = []
    for _ in range(n_frames):
        out.append(K.random_bits(rng, int(rng.integers(*noise_bits))))
        out.append(to_bits(start) + to_bits(rand_bytes(rng, int(rng.integers(*payload)))) + to_bits(end))
    out.append(K.random_bits(rng, int(rng.integers(*noise_bits))))
    return "".join(out)


def make_calls(rng, streams, n_calls, tsc_fail=0.1, max_prefix=24):
    """Split every stream into n_calls rx strings; each call row is a random
    prefix (the bits a TSC strip would drop) + rx, or a failed TSC (-1)."""
    S = len(streams)
    cuts = [np.sort(rng.integers(0, len(s) + 1, n_calls - 1)) for s in streams]
    calls = []
    for c in range(n_calls):
        rows = []
        for s in range(S):
            a = 0 if c == 0 else int(cuts[s][c - 1])
            b = len(streams[s]) if c == n_calls - 1 else int(cuts[s][c])
            rx = streams[s][a:b]
            if rng.random() < tsc_fail:
                rows.append((K.random_bits(rng, int(rng.integers(0, 64))), -1, ""))
            else:
                pre = K.random_bits(rng, int(rng.integers(0, max_prefix)))
                rows.append((pre + rx, len(pre), rx))
        calls.append(rows)
    return calls


def pack_rows(rows):
    nmax = max(len(r[0]) for r in rows)
    stride = (nmax + 7) // 8 + 3          # deliberately not a multiple of 4
    bits = np.zeros((len(rows), stride), np.uint8)
    for s, (row, _, _) in enumerate(rows):
        if row:
            p = Q.pack_bits(row)
            bits[s, : p.size] = p
    nb = np.array([len(r[0]) for r in rows], np.int64)
    off = np.array([r[1] for r in rows], np.int64)
    return bits, nb, off


MARKERS = [(b"\x02", b"\x03"), (b"MESSAGE_START", b"MESSAGE_STOP"), (b"\xA5\x5A", b"\xFF")]


@pytest.mark.parametrize("start,end", MARKERS)
def test_host_framer_matches_string_model(start, end):
    rng = np.random.default_rng(11)
    S = 6
    streams = [make_stream(rng, start, end, 5) for _ in range(S)]
    calls = make_calls(rng, streams, 17)
    fr = Q.Framer(S, start, end)
    refs = [RefFramer() for _ in range(S)]
    n_frames = 0
    for rows in calls:
        bits, nb, off = pack_rows(rows)
        got = fr.push(bits, nb, off, payload_cap=4096)
        for s in range(S):
            exp = refs[s].push(rows[s][2], start, end)
            assert got[s] == exp
            n_frames += bool(exp)
    assert n_frames >= 10


def tad_frames(seed, n_frames, tsc=K.TSC, sps=8, span=8):
    """testAtDataLevel frames (TSC + MESSAGE_START/STOP around the payload text)
    through a seeded ±1 ppm LO pair (testAtDataLevel.cs:27-46)."""
    fs = K.FS
    rs = fs // sps
    tx = O.OracleNCO(100e6, fs, 1, 0, seed=seed)
    rx = O.OracleNCO(100e6, fs, 1, 0, seed=seed + 1)
    return np.concatenate([
        O.apply_lo_pair(tx, rx, O.modulate_text_utf8(fs, rs, K.PAYLOAD + str(i), "MESSAGE_START",
                                                     "MESSAGE_STOP", rrc_alpha=K.ALPHA,
                                                     rrc_span=span, tsc=tsc))
        for i in range(n_frames)])


@pytest.mark.parametrize("tsc,chunks", [(None, 13), (K.TSC, 4000)])
def test_string_model_matches_oracle_framer(tsc, chunks):
    """Pin the string model on the oracle's own DeModulateBytes (C
    restatement, end to end from IQ).  Without a TSC the frames straddle 13
    odd calls; with one, each 4000-sample call keeps what follows its first
    TSC (:413-422)."""
    fs, rs, span = K.FS, K.FS // 8, 8
    sig = tad_frames(15, 10, tsc=tsc or K.TSC)
    a = O.OracleDemod(fs, rs, K.ALPHA, span, tsc=tsc)
    b = O.OracleDemod(fs, rs, K.ALPHA, span, tsc=tsc)
    ref = RefFramer()
    n = sig.size // 2
    if tsc is None:
        spans = [(c[0], c[-1] + 1) for c in np.array_split(np.arange(n), chunks)]
    else:
        spans = [(a0, a0 + chunks) for a0 in range(0, n - chunks + 1, chunks)]
    got = 0
    for lo, hi in spans:
        x = sig[2 * lo: 2 * hi]
        rxb = a.DeModulate(x)
        exp = b.DeModulateBytes(x, b"MESSAGE_START", b"MESSAGE_STOP")
        assert ref.push(rxb, b"MESSAGE_START", b"MESSAGE_STOP") == exp
        got += bool(exp)
    assert got >= 4


# ---------------------------------------------------------------------------
# device framer / TSC (HIP)

@pytest.fixture(scope="module")
def torch_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need an MI355X")
    return torch


RING = 1 << 20   # per-stream ring for the synthetic cases (no frame comes near it)


def run_device(torch, calls, start, end, ring_capacity=RING, payload_cap=4096,
               marker_schedule=None):
    S = len(calls[0])
    fr = Q.DeviceFramer(S, start, end, ring_capacity=ring_capacity)
    # a real stream: handle 0 (torch's legacy default) would mean "library-owned"
    stream = torch.cuda.Stream()
    fr.set_stream(stream.cuda_stream)
    with torch.cuda.stream(stream):
        return _run_device(torch, fr, calls, payload_cap, marker_schedule), fr


def _run_device(torch, fr, calls, payload_cap, marker_schedule):
    S = len(calls[0])
    pay = torch.zeros((S, payload_cap), dtype=torch.uint8, device="cuda")
    npay = torch.zeros(S, dtype=torch.int64, device="cuda")
    outs = []
    for ci, rows in enumerate(calls):
        if marker_schedule:
            fr.set_markers(*marker_schedule[ci])
        bits, nb, off = pack_rows(rows)
        bd = torch.from_numpy(bits).cuda()
        nbd = torch.from_numpy(nb).cuda()
        offd = torch.from_numpy(off).cuda()
        fr.push(bd, nbd, pay, npay, offd)
        n = npay.cpu().numpy()
        p = pay.cpu().numpy()
        outs.append([(int(n[s]), bytes(p[s, : min(int(n[s]), payload_cap)])) for s in range(S)])
    return outs


@pytest.mark.gpu
@pytest.mark.parametrize("start,end", MARKERS)
def test_device_framer_matches_string_model(torch_gpu, start, end):
    rng = np.random.default_rng(21)
    S = 40
    streams = [make_stream(rng, start, end, 6, payload=(0, 300)) for _ in range(S)]
    calls = make_calls(rng, streams, 19)
    outs, _ = run_device(torch_gpu, calls, start, end)
    refs = [RefFramer(RING) for _ in range(S)]
    n_frames = 0
    for ci, rows in enumerate(calls):
        for s in range(S):
            exp = refs[s].push(rows[s][2], start, end)
            n, got = outs[ci][s]
            assert (n, got) == (len(exp), exp), (ci, s)
            n_frames += bool(exp)
    assert n_frames >= 2 * S


@pytest.mark.gpu
def test_device_framer_long_rows_and_offsets(torch_gpu):
    """Rows of ~260k bits (one C2 call's worth) with frames of every lock
    offset and a payload longer than the caller's payload buffer."""
    rng = np.random.default_rng(22)
    start, end = b"MESSAGE_START", b"MESSAGE_STOP"
    S = 8
    streams = [make_stream(rng, start, end, 8, noise_bits=(0, 60000), payload=(0, 3000))
               for _ in range(S)]
    calls = make_calls(rng, streams, 4, tsc_fail=0.0, max_prefix=64)
    outs, _ = run_device(torch_gpu, calls, start, end, payload_cap=1024)
    refs = [RefFramer(RING) for _ in range(S)]
    for ci, rows in enumerate(calls):
        for s in range(S):
            exp = refs[s].push(rows[s][2], start, end)
            n, got = outs[ci][s]
            assert n == len(exp) and got == exp[:1024], (ci, s)


@pytest.mark.gpu
def test_device_framer_overflow_and_marker_change(torch_gpu):
    rng = np.random.default_rng(23)
    S = 16
    m1, m2 = (b"\x02", b"\x03"), (b"\xA5\x5A", b"\xFF")
    streams = [make_stream(rng, m1[0], m1[1], 4, payload=(0, 60)) +
               make_stream(rng, m2[0], m2[1], 4, payload=(0, 60)) for _ in range(S)]
    calls = make_calls(rng, streams, 12)
    sched = [m1] * 6 + [m2] * 6
    outs, fr = run_device(torch_gpu, calls, *m1, ring_capacity=24, marker_schedule=sched)
    refs = [RefFramer(ring_capacity=24) for _ in range(S)]
    for ci, rows in enumerate(calls):
        for s in range(S):
            exp = refs[s].push(rows[s][2], *sched[ci])
            assert outs[ci][s] == (len(exp), exp), (ci, s)
    inf, cnt, car = fr.status()
    for s in range(S):
        assert bool(inf[s]) == refs[s].in_frame
        assert cnt[s] == len(refs[s].ring)
        assert car[s] == len(refs[s].carry)


@pytest.mark.gpu
@pytest.mark.parametrize("tsc", [K.TSC, "1011001", "1" * 33, K.TSC * 3, "01" * 2100, "   ", "10x1"])
def test_tsc_find_device_matches_str_find(torch_gpu, tsc):
    torch = torch_gpu
    rng = np.random.default_rng(24)
    S = 33
    rows = []
    for s in range(S):
        r = K.random_bits(rng, int(rng.integers(0, 5000)))
        if s % 3 and tsc.strip() and set(tsc) <= {"0", "1"}:   # bit rows hold only 0/1
            i = int(rng.integers(0, len(r) + 1))
            r = r[:i] + tsc + r[i:] + K.random_bits(rng, int(rng.integers(0, 100)))
        rows.append(r)
    bits, nb, _ = pack_rows([(r, 0, r) for r in rows])
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        offs = torch.full((S,), -7, dtype=torch.int64, device="cuda")
        bd = torch.from_numpy(bits).cuda()
        Q.tsc_find_device(bd, torch.from_numpy(nb).cuda(), tsc, offs, st.cuda_stream)
        got = offs.cpu().numpy()
    for s, r in enumerate(rows):
        if not tsc.strip():
            exp = 0
        else:
            i = r.find(tsc)
            exp = -1 if i < 0 else i + len(tsc)
        assert got[s] == exp, (s, len(r))
        assert Q.tsc_find(bits[s], len(r), tsc) == exp


@pytest.mark.gpu
def test_device_bytes_chain_matches_oracle(torch_gpu):
    """DeModulateBytes end to end on the device: process_device -> TSC search
    -> device framer, per stream against the oracle's DeModulateBytes on the
    testAtDataLevel frames (TSC + MESSAGE_START/STOP) with per-stream LOs."""
    torch = torch_gpu
    fs, sps, span = K.FS, 8, 8
    rs = fs // sps
    S = 4
    sigs = [tad_frames(30 + 2 * s, 10) for s in range(S)]
    n_all = min(x.size // 2 for x in sigs)
    chunk = 4000
    p = Q.params(fs, rs, K.ALPHA, span, max_samples_per_call=chunk)
    dm = Q.BatchDemodulator(S, p)
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    dm.set_stream(st.cuda_stream)
    fr = Q.DeviceFramer(S, b"MESSAGE_START", b"MESSAGE_STOP")
    fr.set_stream(st.cuda_stream)
    ms = dm.max_symbols(chunk)
    bits = torch.zeros((S, (2 * ms + 7) // 8 + 8), dtype=torch.uint8, device="cuda")
    nbits = torch.zeros(S, dtype=torch.int64, device="cuda")
    offs = torch.zeros(S, dtype=torch.int64, device="cuda")
    pay = torch.zeros((S, 256), dtype=torch.uint8, device="cuda")
    npay = torch.zeros(S, dtype=torch.int64, device="cuda")
    orc = [O.OracleDemod(fs, rs, K.ALPHA, span, tsc=K.TSC) for _ in range(S)]
    frames = 0
    for a in range(0, n_all - chunk + 1, chunk):
        x = np.stack([sig[2 * a: 2 * (a + chunk)] for sig in sigs]).astype(np.float32)
        xd = torch.from_numpy(x).cuda()
        dm.process_device(xd, chunk, bits, nbits)
        Q.tsc_find_device(bits, nbits, K.TSC, offs, st.cuda_stream)
        fr.push(bits, nbits, pay, npay, offs)
        n = npay.cpu().numpy()
        pb = pay.cpu().numpy()
        for s in range(S):
            exp = orc[s].DeModulateBytes(x[s], b"MESSAGE_START", b"MESSAGE_STOP")
            assert (int(n[s]), bytes(pb[s, : int(n[s])])) == (len(exp), exp), (a, s)
            frames += bool(exp)
    torch.cuda.set_stream(torch.cuda.default_stream())
    assert frames >= 2 * S
