"""The multi-GPU group behind the C ABI (qpsk_demod_group_*).

Per-instance state is what makes a batch split exact: each reference
QPSKDeModulator owns its FIR / M&M / Costas / differential state
(QPSKDeModulator.cs:20-73), so a shard of streams on its own handle computes
exactly what the same streams compute inside one handle.

CPU: the shard arithmetic (qpsk_shard_streams equals bench.py's rank split and
covers every stream once) and the argument checks that run before any device
is touched.  GPU: a group of two shards on device 0 against one handle over
the same batch, bits and symbols bit for bit, over ragged consecutive calls,
host and device memory, and a per-shard state round trip.
"""
import ctypes as C
import os
import sys

import numpy as np
import pytest

import common as K
import oracle as O
import qpsk_amd as Q

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.argv = sys.argv[:1]
import bench  # noqa: E402


@pytest.mark.parametrize("S,n", [(1, 1), (5, 2), (7, 3), (256, 8), (4096, 8), (32768, 8), (10, 7), (3, 3)])
def test_shard_streams_matches_rank_split(S, n):
    covered = []
    for k in range(n):
        f, c = Q.shard_streams(S, n, k)
        lo, hi = bench.shard_streams(S, k, n)
        assert (f, c) == (lo, hi - lo)
        covered += list(range(f, f + c))
    assert covered == list(range(S))


def test_shard_streams_rejects_bad_arguments():
    L = Q.lib()
    f, c = C.c_int32(), C.c_int32()
    assert L.qpsk_shard_streams(10, 0, 0, C.byref(f), C.byref(c)) == Q.QPSK_ERR_ARGUMENT
    assert L.qpsk_shard_streams(10, 2, 2, C.byref(f), C.byref(c)) == Q.QPSK_ERR_ARGUMENT
    assert L.qpsk_shard_streams(-1, 2, 0, C.byref(f), C.byref(c)) == Q.QPSK_ERR_ARGUMENT
    assert L.qpsk_shard_streams(10, 2, 0, None, C.byref(c)) == Q.QPSK_ERR_ARGUMENT_NULL


def test_group_create_checks_arguments_before_any_device():
    L = Q.lib()
    p = Q.params(K.FS, K.FS // 8, K.ALPHA, 8)
    g = C.c_void_p()
    devs = (C.c_int32 * 2)(0, 0)
    assert L.qpsk_demod_group_create(C.byref(p), devs, 2, 1, C.byref(g)) == Q.QPSK_ERR_ARGUMENT   # empty shard
    assert L.qpsk_demod_group_create(C.byref(p), devs, 0, 4, C.byref(g)) == Q.QPSK_ERR_ARGUMENT
    assert L.qpsk_demod_group_create(C.byref(p), None, 2, 4, C.byref(g)) == Q.QPSK_ERR_ARGUMENT_NULL
    bad = (C.c_int32 * 2)(0, -1)
    assert L.qpsk_demod_group_create(C.byref(p), bad, 2, 4, C.byref(g)) == Q.QPSK_ERR_ARGUMENT
    assert g.value is None
    assert L.qpsk_demod_group_destroy(None) == 0
    assert L.qpsk_demod_group_size(None) == Q.QPSK_ERR_ARGUMENT_NULL
    assert L.qpsk_demod_group_state_bytes(None, 0) == 0


# ---------------------------------------------------------------------------
# GPU: group of two shards on device 0 == one handle, bit for bit
# ---------------------------------------------------------------------------
def _ragged_calls(S, n, rng):
    calls, used = [], np.zeros(S, np.int64)
    for c in range(4):
        lens = np.full(S, 1000) if c == 0 else rng.integers(0, n // 5, S)
        if c == 2:
            lens[: S // 2] = 0                     # a whole shard with empty calls
        calls.append(lens.astype(np.int64))
        used += lens
    calls.append((n - used).astype(np.int64))
    return calls


def _rows_of_call(iq, pos, lens):
    S = iq.shape[0]
    n = int(lens.max())
    x = np.zeros((S, 2 * max(n, 1)), np.float32)
    for s in range(S):
        x[s, : 2 * lens[s]] = iq[s, 2 * pos[s]: 2 * (pos[s] + lens[s])]
    return x[:, : 2 * n]


@pytest.mark.gpu
@pytest.mark.parametrize("sps,span,S", [(8, 8, 7), (4, 32, 6)])
def test_group_two_shards_equal_one_handle_host_memory(sps, span, S):
    iq = K.batch_signals(S, seed0=900 + sps, sps=sps, span=span, n_bits=2400, snr_db=15)
    n = iq.shape[1] // 2
    calls = _ragged_calls(S, n, np.random.default_rng(sps))
    p = Q.params(K.FS, K.FS // sps, K.ALPHA, span, max_samples_per_call=n)
    one = Q.BatchDemodulator(S, p)
    grp = Q.DemodGroup(S, p, [0, 0])
    assert grp.size() == 2
    f1, c1, d1, _ = grp.shard(1)
    assert (f1, c1, d1) == (S // 2, S - S // 2, 0)
    pos = np.zeros(S, np.int64)
    last = S - 1          # the second shard's last stream
    rows_last = []
    for ci, lens in enumerate(calls):
        x = _rows_of_call(iq, pos, lens)
        a = one.process(x, lengths=lens, want_syms=True)
        b = grp.process(x, lengths=lens, want_syms=True)
        rows_last.append((Q.unpack_bits(b[0][last], int(b[1][last])), b[2][last, : 2 * int(b[3][last])].copy()))
        assert np.array_equal(a[1], b[1]) and np.array_equal(a[3], b[3]), f"call {ci}: counts"
        for s in range(S):
            nb, ns = int(a[1][s]), int(a[3][s])
            assert np.array_equal(a[0][s, : (nb + 7) // 8], b[0][s, : (nb + 7) // 8]), (ci, s)
            assert K.bitwise_equal(a[2][s, : 2 * ns], b[2][s, : 2 * ns]), (ci, s)
        pos += lens
    # deModulateConstellation through the group
    x = iq[:, : 2 * 3000]
    a = one.process(x, mode=Q.MODE_CONSTELLATION)
    b = grp.process(x, mode=Q.MODE_CONSTELLATION)
    for s in range(S):
        ns = int(a[3][s])
        assert int(b[3][s]) == ns and K.bitwise_equal(a[2][s, : 2 * ns], b[2][s, : 2 * ns])
    # and the second shard's last stream is the oracle's, call for call
    d = K.oracle_for(sps, span)
    pos = 0
    for ci, lens in enumerate(calls):
        rb, rs, _ = d.demodulate_ex(iq[last, 2 * pos: 2 * (pos + lens[last])])
        assert rows_last[ci][0] == rb and K.bitwise_equal(rows_last[ci][1], rs), f"call {ci}"
        pos += int(lens[last])
    one.close()
    grp.close()


@pytest.mark.gpu
def test_group_device_memory_and_shard_state_round_trip():
    import torch
    sps, span, S, n = 8, 8, 9, 6000
    dev = torch.device("cuda", 0)
    iq, _ = Q.synth_generate(S, 2 * n, K.FS, K.FS // sps, rrc_alpha=K.ALPHA, rrc_span=span, seed=31, lo_ppm=1.0)
    p = Q.params(K.FS, K.FS // sps, K.ALPHA, span, max_samples_per_call=n)
    one = Q.BatchDemodulator(S, p)
    grp = Q.DemodGroup(S, p, [0, 0, 0])
    ms = one.max_symbols(n)

    def out():
        return (torch.zeros((S, (2 * ms + 7) // 8 + 8), dtype=torch.uint8, device=dev),
                torch.zeros(S, dtype=torch.int64, device=dev),
                torch.zeros((S, 2 * ms), dtype=torch.float32, device=dev),
                torch.zeros(S, dtype=torch.int64, device=dev))
    x0, x1 = iq[:, : 2 * n].contiguous(), iq[:, 2 * n:].contiguous()
    # every output zeroed up front on torch's stream, which the handles'
    # library-owned streams do not follow
    a, b, c, e, r = out(), out(), out(), out(), out()
    torch.cuda.synchronize(dev)
    one.process_device(x0, n, a[0], a[1], syms_dev=a[2], n_syms_dev=a[3])
    torch.cuda.synchronize(dev)
    grp.process_device(x0, n, b[0], b[1], syms_dev=b[2], n_syms_dev=b[3])   # joined on return
    states = [grp.get_state(k) for k in range(3)]
    # the second call twice on the group: once straight on, once after a
    # restore of every shard's state blob -- identical rows
    grp.process_device(x1, n, c[0], c[1], syms_dev=c[2], n_syms_dev=c[3])
    for k in range(3):
        grp.set_state(k, states[k])
    grp.process_device(x1, n, e[0], e[1], syms_dev=e[2], n_syms_dev=e[3])
    one.process_device(x1, n, r[0], r[1], syms_dev=r[2], n_syms_dev=r[3])
    torch.cuda.synchronize(dev)
    for ref, got in ((a, b), (r, c), (r, e)):
        assert torch.equal(ref[1], got[1]) and torch.equal(ref[3], got[3])
        for s in range(S):
            nb, ns = int(ref[1][s]), int(ref[3][s])
            assert torch.equal(ref[0][s, : (nb + 7) // 8], got[0][s, : (nb + 7) // 8]), s
            assert torch.equal(ref[2][s, : 2 * ns].view(torch.int32), got[2][s, : 2 * ns].view(torch.int32)), s
    # a shard's blob does not fit another shard's handle (3 + 3 + 3 streams fit; 9 in one do not)
    with pytest.raises(ValueError):
        one.set_state(states[0])
    one.close()
    grp.close()


@pytest.mark.gpu
def test_group_rejects_bad_rows_before_any_shard_runs():
    sps, span, S = 8, 8, 4
    p = Q.params(K.FS, K.FS // sps, K.ALPHA, span, max_samples_per_call=4096)
    grp = Q.DemodGroup(S, p, [0, 0])
    before = [grp.get_state(k) for k in range(2)]
    L = Q.lib()
    x = np.zeros((S, 2 * 4096), np.float32)
    nb = np.zeros(S, np.int64)
    bits = np.zeros((S, 4), np.uint8)                  # rows far too short for 4096 samples
    rc = L.qpsk_demod_group_process(grp._g, 0, x.ctypes.data, x.shape[1], 4096, None, Q.MEM_HOST,
                                    bits.ctypes.data, 4, nb.ctypes.data, None, 0, None)
    assert rc == Q.QPSK_ERR_ARGUMENT
    assert [grp.get_state(k) for k in range(2)] == before
    grp.close()
