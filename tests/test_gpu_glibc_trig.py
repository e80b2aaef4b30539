"""GPU parity with the Costas NCO on glibc's own sin / cos
(qpsk_demod_params.costas_trig = 1, csrc/qpsk_glibc_trig.h).

.NET's Math.Sin / Math.Cos (CostasLoopQpsk.cs:69-70) are glibc's double sin
and cos on a Linux x86-64 host; the oracle's TRIG_LIBM mode calls that libm.
With costas_trig = 1 the GPU evaluates the same algorithm operation for
operation (tools/check_glibc_sin.c: 680M arguments, 0 differences from
libm), so bits AND rotated symbols must be bit-identical to the libm oracle
-- no tolerance -- in every mode, including the |theta| >= 105414350
Payne-Hanek reduction a QPSK false lock reaches.
"""
import numpy as np
import pytest

import common as K
import oracle as O
import qpsk_amd as Q
from test_gpu_parity import assert_same, async_run, gpu_run, oracle_run

pytestmark = pytest.mark.gpu

LIBM = dict(trig=O.TRIG_LIBM)
GL = dict(costas_trig=1)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need an MI355X")
    yield


@pytest.mark.parametrize("sps,span", K.CONFIGS)
def test_glibc_trig_single_call_bit_exact(sps, span):
    iq = K.batch_signals(5, seed0=900, sps=sps, span=span, n_bits=3000, snr_db=16)
    calls = [[iq.shape[1] // 2] * 5]
    assert_same(gpu_run(iq, calls, sps, span, **GL), oracle_run(iq, calls, sps, span, **LIBM))


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 6, 7])
def test_glibc_trig_ragged_chunks_every_loop_shape(variant):
    sps, span = 8, 8
    iq = K.batch_signals(4, seed0=910, sps=sps, span=span, n_bits=4000, snr_db=14)
    n = iq.shape[1] // 2
    rng = np.random.default_rng(variant)
    calls, used = [], np.zeros(4, np.int64)
    for _ in range(4):
        lens = rng.integers(0, n // 5, 4)
        calls.append([int(v) for v in lens])
        used += lens
    calls.append([int(n - u) for u in used])
    got = gpu_run(iq, calls, sps, span, loop_variant=variant, **GL)
    assert_same(got, oracle_run(iq, calls, sps, span, **LIBM))


@pytest.mark.parametrize("fll", [False, True])
def test_glibc_trig_pipelined_bit_exact(fll):
    kw = dict(enable_fll=True, cfo_loop_bandwidth=1e-3) if fll else {}
    okw = dict(enable_fll=True, cfo_loop_bw=1e-3) if fll else {}
    iq = K.batch_signals(5, seed0=920, sps=8, span=8, n_bits=2400, snr_db=16, cfo_hz=3000.0 if fll else 0.0,
                         multipath=fll)
    n = iq.shape[1] // 2
    calls = [[n // 4] * 5, [n // 3] * 5, [n - n // 4 - n // 3] * 5]
    got, _ = async_run(iq, calls, 8, 8, **GL, **kw)
    assert_same(got, oracle_run(iq, calls, 8, 8, **LIBM, **okw))


def test_glibc_trig_constellation_and_nondifferential():
    iq = K.batch_signals(3, seed0=930, sps=4, span=32, n_bits=2000, snr_db=16)
    n = iq.shape[1] // 2
    calls = [[n // 2] * 3, [n - n // 2] * 3]
    mode = [Q.MODE_CONSTELLATION, Q.MODE_DEMODULATE]
    assert_same(gpu_run(iq, calls, 4, 32, mode=mode, **GL), oracle_run(iq, calls, 4, 32, mode=mode, **LIBM))
    iq = K.batch_signals(3, seed0=931, sps=8, span=8, n_bits=2000, snr_db=16, differential=False)
    calls = [[iq.shape[1] // 2] * 3]
    assert_same(gpu_run(iq, calls, 8, 8, differential=False, **GL),
                oracle_run(iq, calls, 8, 8, differential=False, **LIBM))


def test_glibc_trig_huge_theta_payne_hanek():
    """Samples scaled by 1e12: the first phase error moves freq by ~1e10, so
    theta passes 105414350 at once and every symbol after takes glibc's
    __branred reduction; symbols stay bit-identical to the libm oracle."""
    iq = K.batch_signals(3, seed0=940, sps=8, span=8, n_bits=800, snr_db=20) * np.float32(1e12)
    n = iq.shape[1] // 2
    calls = [[n // 3] * 3, [n - n // 3] * 3]
    got, ref = gpu_run(iq, calls, 8, 8, **GL), oracle_run(iq, calls, 8, 8, **LIBM)
    for ci, (ra, rb) in enumerate(zip(got, ref)):
        for s, ((ba, sa), (bb, sb)) in enumerate(zip(ra, rb)):
            assert ba == bb, f"call {ci} stream {s}: bits differ"
            assert np.array_equal(sa.view(np.uint32), sb.view(np.uint32)), f"call {ci} stream {s}"


def test_glibc_trig_rejects_unknown_mode():
    with pytest.raises(ValueError):
        Q.BatchDemodulator(1, Q.params(K.FS, K.FS // 8, K.ALPHA, 8, costas_trig=2))
