"""CPU checks of the drop-in boundary (no GPU needed).

* libqpsk_demod.so loads and exports every entry point include/qpsk_demod.h declares;
* the constructor math (RRC taps, loop gains, FLL taps, validation) equals the
  oracle's, i.e. the reference ctor (QPSKDeModulator.cs:11-56);
* the host framer (DeModulateBytes state machine) and TSC search equal the
  oracle on the same bits;
* the product's portable sincos header equals the oracle's copy bit for bit.
"""
import os
import re
import subprocess

import numpy as np
import pytest

import common as K
import oracle as O
import qpsk_amd as Q

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "qpsk_demod.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(qpsk_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    names = header_functions()
    assert len(names) >= 20
    L = Q.lib()
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(Q.EXPORTED_SYMBOLS)
    out = subprocess.check_output(["nm", "-D", "--defined-only", Q.LIB_PATH]).decode()
    for n in names:
        assert re.search(r"\bT " + n + r"\b", out), n
    assert L.qpsk_abi_version() == 3


def test_library_has_gfx950_code_object():
    blob = open(Q.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


@pytest.mark.parametrize("sps,span,alpha", [(8, 8, K.ALPHA), (4, 32, K.ALPHA), (2, 10, K.ALPHA),
                                            (2, 6, 0.9), (3, 5, 0.35), (2, 8, 0.1)])
def test_design_matches_oracle(sps, span, alpha):
    fs, rs = K.FS, K.FS // sps
    taps, gains, lo, up = Q.design(Q.params(fs, rs, alpha, span))
    dm = O.OracleDemod(fs, rs, alpha, span)
    assert np.array_equal(taps, dm.rrc_f32())
    og = dm.gains()
    for k in og:
        assert gains[k] == og[k], k
    of = O.OracleFLL(np.float32(fs // rs), np.float32(alpha), 40, np.float32(np.float32(1e-4)))
    olo, oup = of.taps()
    assert np.array_equal(lo, olo) and np.array_equal(up, oup)


def test_design_reference_values():
    """SURVEY.md §8 constants for the default loop bandwidths."""
    _, g, _, _ = Q.design(Q.params(K.FS, K.FS // 8, K.ALPHA, 8))
    assert abs(g["kp"] - 2.6225e-3) < 1e-7 and abs(g["ki"] - 3.4432e-6) < 1e-10
    assert abs(g["costas_alpha"] - 0.137516) < 1e-6 and abs(g["costas_beta"] - 0.0101843) < 1e-7


@pytest.mark.parametrize("kw", [dict(symbol_rate=2 * K.FS), dict(rrc_alpha=1.5),
                                dict(rrc_alpha=-0.1), dict(cfo_loop_bandwidth=0.0)])
def test_ctor_validation_maps_to_out_of_range(kw):
    args = dict(sample_rate=K.FS, symbol_rate=K.FS // 8, rrc_alpha=0.4, rrc_span=8)
    args.update(kw)
    with pytest.raises(ValueError):
        Q.design(Q.params(**args))
    assert Q.lib().qpsk_demod_design(Q.params(**args), None, 0, None, None, None) == Q.QPSK_ERR_OUT_OF_RANGE


def _oracle_call_bits(dm, x):
    bits, _, tsc_idx = dm.demodulate_ex(x)
    return bits, tsc_idx


def test_framer_and_tsc_match_oracle():
    """Frames of testAtDataLevel fed in odd chunks: the product framer, fed the
    oracle's per-call bits, must return exactly what the oracle's own
    DeModulateBytes returns."""
    fs, rs, span = K.FS, K.FS // 8, 8
    frames = []
    tx = O.OracleNCO(100e6, fs, 1, 0, seed=5)
    rx = O.OracleNCO(100e6, fs, 1, 0, seed=6)
    for i in range(6):
        sig = O.modulate_text_utf8(fs, rs, K.PAYLOAD + str(i), "MESSAGE_START", "MESSAGE_STOP",
                                   rrc_alpha=K.ALPHA, rrc_span=span, tsc=K.TSC)
        frames.append(O.apply_lo_pair(tx, rx, sig))
    stream = np.concatenate(frames)
    chunks = np.array_split(np.arange(stream.size // 2), 23)
    a = O.OracleDemod(fs, rs, K.ALPHA, span)        # bits source
    b = O.OracleDemod(fs, rs, K.ALPHA, span)        # reference framer
    fr = Q.Framer(1, b"MESSAGE_START", b"MESSAGE_STOP")
    got_any = 0
    for c in chunks:
        x = stream.reshape(-1, 2)[c].reshape(-1)
        bits, _ = _oracle_call_bits(a, x)
        exp = b.DeModulateBytes(x, b"MESSAGE_START", b"MESSAGE_STOP")
        packed = Q.pack_bits(bits) if bits else np.zeros(1, np.uint8)
        out = fr.push(packed[None, :], np.array([len(bits)]))[0]
        assert out == exp
        got_any += bool(out)
    assert got_any >= 3


def test_framer_overflow_resync():
    bits = K.random_bits(np.random.default_rng(1), 400)
    start, end = b"\x02", b"\x03"
    s_bits = "".join(format(v, "08b") for v in start)
    stream = s_bits + bits
    fr = Q.Framer(1, start, end, ring_capacity=8)
    p = Q.pack_bits(stream)
    out = fr.push(p[None, :], np.array([len(stream)]))
    assert out[0] == b""   # overflowed (more than 8 payload bytes, no end) -> dropped


def test_tsc_find_matches_str_find():
    rng = np.random.default_rng(2)
    for _ in range(20):
        s = K.random_bits(rng, 300) + K.TSC + K.random_bits(rng, 50)
        p = Q.pack_bits(s)
        i = s.find(K.TSC)
        assert Q.tsc_find(p, len(s), K.TSC) == i + len(K.TSC)
    p = Q.pack_bits("0" * 100)
    assert Q.tsc_find(p, 100, K.TSC) == -1
    assert Q.tsc_find(p, 100, "   ") == 0          # IsNullOrWhiteSpace -> no TSC


def test_unpack_pack_roundtrip():
    s = K.random_bits(np.random.default_rng(3), 77)
    assert Q.unpack_bits(Q.pack_bits(s), 77) == s


def test_sincos_headers_bit_identical(tmp_path):
    src = tmp_path / "sc.cpp"
    src.write_text(r'''
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include "or_sincos.h"
#include "qpsk_sincos.h"
int main() {
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> u(-7.0, 7.0), w(-3e6, 3e6);
  long bad = 0;
  for (long i = 0; i < 2000000; ++i) {
    double x = (i % 10 == 0) ? w(g) : u(g);
    double s1, c1, s2, c2; or_sincos(x, &s1, &c1); qpsk_sincos(x, &s2, &c2);
    float fs1, fc1, fs2, fc2; or_sincosf((float)x, &fs1, &fc1); qpsk_sincosf((float)x, &fs2, &fc2);
    if (memcmp(&s1,&s2,8) || memcmp(&c1,&c2,8) || memcmp(&fs1,&fs2,4) || memcmp(&fc1,&fc2,4)) ++bad;
  }
  printf("%ld\n", bad);
  return 0;
}
''')
    exe = tmp_path / "sc"
    subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-mfma", "-I", os.path.join(ROOT, "oracle"),
                           "-I", os.path.join(ROOT, "qpsk-modulator-demodulator_amd", "csrc"),
                           str(src), "-o", str(exe)])
    assert subprocess.check_output([str(exe)]).decode().strip() == "0"


def _header_floats(path, macro):
    import re
    text = open(path).read()
    body = text.split(f"#define {macro} \\", 1)[1].split("#define", 1)[0]
    vals = []
    for tok in re.findall(r"-?0x[0-9a-fA-F.]+p[+-]?\d+f?|-?0\.0f?", body):
        vals.append(float.fromhex(tok.rstrip("f")))
    return vals


def test_sincos_tables_match_independent_model():
    """Product and oracle table headers are identical and equal the table the
    numpy model recomputes on its own (tests/refmodel.py)."""
    import refmodel as RM
    prod = os.path.join(ROOT, "qpsk-modulator-demodulator_amd", "csrc", "qpsk_sincos_table.h")
    orc = os.path.join(ROOT, "oracle", "or_sincos_table.h")
    hi_p, lo_p = _header_floats(prod, "QPSK_SINCOS_TAB_VALUES_HI"), _header_floats(prod, "QPSK_SINCOS_TAB_VALUES_LO")
    hi_o, lo_o = _header_floats(orc, "OR_SINCOS_TAB_VALUES_HI"), _header_floats(orc, "OR_SINCOS_TAB_VALUES_LO")
    assert hi_p == hi_o and lo_p == lo_o and len(hi_p) == 1024 and len(lo_p) == 1024
    ref = [v for ts, ls, tc, lc in RM.SINCOS_TABLE for v in (ts, tc)]
    ref_lo = [v for ts, ls, tc, lc in RM.SINCOS_TABLE for v in (ls, lc)]
    assert hi_p == ref and lo_p == ref_lo


@pytest.mark.parametrize("kw", [dict(loop_variant=8), dict(loop_variant=-1), dict(vector_lanes=3),
                                dict(max_samples_per_call=0)])
def test_create_rejects_bad_knobs_before_touching_a_device(kw):
    """Argument checks run before any HIP call, so they hold on a CPU-only host."""
    import ctypes as C
    args = dict(sample_rate=K.FS, symbol_rate=K.FS // 8, rrc_alpha=0.4, rrc_span=8)
    args.update(kw)
    h = C.c_void_p()
    assert Q.lib().qpsk_demod_create(C.byref(Q.params(**args)), 4, C.byref(h)) == Q.QPSK_ERR_ARGUMENT


GATE_ENV = ["QPSK_PIPELINE_GATE", "AMD_SERIALIZE_KERNEL", "AMD_SERIALIZE_COPY", "HIP_LAUNCH_BLOCKING",
            "CUDA_LAUNCH_BLOCKING", "ROCPROF_COUNTER_COLLECTION", "ROCPROFILER_KERNEL_SERIALIZATION",
            "HSA_ENABLE_DEBUG"]


@pytest.mark.parametrize("env,want", [
    ({}, 1),
    ({"QPSK_PIPELINE_GATE": "0"}, 0),
    ({"QPSK_PIPELINE_GATE": "1", "AMD_SERIALIZE_KERNEL": "3"}, 1),   # explicit opt-in wins
    ({"AMD_SERIALIZE_KERNEL": "1"}, 0),
    ({"AMD_SERIALIZE_KERNEL": "3"}, 0),
    ({"AMD_SERIALIZE_KERNEL": "0"}, 1),
    ({"AMD_SERIALIZE_COPY": "2"}, 0),
    ({"HIP_LAUNCH_BLOCKING": "1"}, 0),
    ({"HIP_LAUNCH_BLOCKING": "0"}, 1),
    ({"CUDA_LAUNCH_BLOCKING": "1"}, 0),
    ({"ROCPROF_COUNTER_COLLECTION": "1"}, 0),
    ({"ROCPROF_COUNTER_COLLECTION": "0"}, 1),
    ({"ROCPROFILER_KERNEL_SERIALIZATION": "1"}, 0),
    ({"HSA_ENABLE_DEBUG": "1"}, 0),
    ({"AMD_SERIALIZE_KERNEL": ""}, 1),   # set but empty = unset
])
def test_pipeline_gate_predicate(monkeypatch, env, want):
    """The residency gate (qpsk_runtime.hip, process_async_one) parks the FIR's
    stream on hipStreamWaitValue64 with no timeout, so it must be off wherever
    dispatch is serialised (include/qpsk_demod.h, qpsk_pipeline_gate_enabled);
    evaluated without a device."""
    for k in GATE_ENV:
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    assert Q.lib().qpsk_pipeline_gate_enabled() == want


@pytest.mark.parametrize("requested,S,sps,cus,want", [
    (0, 256, 8.0, 256, 7),      # C2: 43 workgroups of 6 x 512
    (0, 1536, 8.0, 256, 7),     # 256 workgroups: still one pass
    (0, 1537, 8.0, 256, 6),     # 12 x 256
    (0, 2048, 8.0, 256, 6),
    (0, 3072, 8.0, 256, 6),
    (0, 3073, 8.0, 256, 0),     # 24 x 128 would need 129 > cus / 2 workgroups
    (0, 4096, 8.0, 256, 0),     # C4 shard: the 32 x 64 default
    (0, 8192, 8.0, 256, 0),     # C5
    (0, 3073, 8.0, 1024, 7),    # a larger chip keeps the long rounds
    (0, 256, 4.0, 256, 0),      # sps < 8 (C3): the launcher's default
    (0, 256, 7.99, 256, 0),
    (0, 256, 30.0, 256, 7),     # the reference's testFullDemodChain sps
    (2, 256, 8.0, 256, 2),      # an explicit shape is kept
    (0, 256, 8.0, 0, 0),        # unknown CU count
])
def test_auto_loop_shape(requested, S, sps, cus, want):
    """The loop shape qpsk_demod_create picks (long rounds with
    shadow lanes while they fit the chip in one pass, A/B-measured at 256,
    1024, 2048 and 4096 streams); evaluated without a device."""
    assert Q.lib().qpsk_demod_pick_loop_variant(requested, S, sps, cus) == want
