"""ctypes wrapper around the CPU oracle (liboracle.so).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker.  The product library never loads
it.  Parity with the C# reference is unpinned (no .NET runtime, no golden
vectors in the reference); see qpsk_oracle.h and DESIGN.md.

Mirrors the reference classes:
  QPSKDeModulator  -> OracleDemod     (QPSKDeModulator.cs:11-457)
  ComplexFIRFilter -> oracle_fir      (FIRFilter.cs:8-232)
  MuellerMuller    -> OracleMM        (MuellerMuller.cs:17-249)
  CostasLoopQpsk   -> OracleCostas    (CostasLoopQpsk.cs:19-130)
  FLLBandEdgeFilter-> OracleFLL       (Band-Edge Filter.cs:14-203)
  QPSKModulator    -> modulate()      (QPSKModulator.cs:104-167)
  NCO              -> OracleNCO       (LocalOscilator.cs:5-194)
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

TRIG_LIBM = 0
TRIG_PORTABLE = 1

_f32p = C.POINTER(C.c_float)
_f64p = C.POINTER(C.c_double)
_u8p = C.POINTER(C.c_uint8)
_i64p = C.POINTER(C.c_long)


class DemodCfg(C.Structure):
    _fields_ = [
        ("sample_rate", C.c_int),
        ("symbol_rate", C.c_int),
        ("rrc_alpha", C.c_float),
        ("rrc_span", C.c_int),
        ("symbol_sync_bw", C.c_double),
        ("costas_loop_bw", C.c_double),
        ("cfo_loop_bw", C.c_double),
        ("differential", C.c_int),
        ("tsc", C.c_char_p),
        ("enable_fll", C.c_int),
        ("lanes", C.c_int),
        ("trig_mode", C.c_int),
        ("ring_capacity", C.c_long),
        ("iq_balance", C.c_int),
    ]


class IQB(C.Structure):
    _fields_ = [("avg_re", C.c_float), ("avg_im", C.c_float)]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.or_rrc_taps.argtypes = [C.c_double, C.c_double, C.c_int, C.c_int, _f64p, C.c_int]
        L.or_rrc_taps.restype = C.c_int
        L.or_cfir_new.argtypes = [_f32p, C.c_int, C.c_int]
        L.or_cfir_new.restype = C.c_void_p
        L.or_cfir_free.argtypes = [C.c_void_p]
        L.or_cfir_filter.argtypes = [C.c_void_p, _f32p, _f32p, C.c_long]
        L.or_mm_new.argtypes = [C.c_double, C.c_double, C.c_double]
        L.or_mm_new.restype = C.c_void_p
        L.or_mm_free.argtypes = [C.c_void_p]
        L.or_mm_process.argtypes = [C.c_void_p, _f32p, C.c_long, _f32p, C.c_long]
        L.or_mm_process.restype = C.c_long
        L.or_costas_new.argtypes = [C.c_double, C.c_double, C.c_double, C.c_int]
        L.or_costas_new.restype = C.c_void_p
        L.or_costas_free.argtypes = [C.c_void_p]
        L.or_costas_process.argtypes = [C.c_void_p, C.c_float, C.c_float, _f32p, _f32p]
        L.or_costas_state.argtypes = [C.c_void_p, _f64p, _f64p]
        L.or_fll_new.argtypes = [C.c_float, C.c_float, C.c_int, C.c_float, C.c_int, C.c_int]
        L.or_fll_new.restype = C.c_void_p
        L.or_fll_free.argtypes = [C.c_void_p]
        L.or_fll_process.argtypes = [C.c_void_p, _f32p, _f32p, C.c_long]
        L.or_fll_taps.argtypes = [C.c_void_p, _f32p, _f32p, C.c_int]
        L.or_fll_taps.restype = C.c_int
        L.or_fll_state.argtypes = [C.c_void_p, _f32p, _f32p]
        L.or_demod_cfg_default.argtypes = [C.POINTER(DemodCfg), C.c_int, C.c_int]
        L.or_demod_new.argtypes = [C.POINTER(DemodCfg), C.POINTER(C.c_int)]
        L.or_demod_new.restype = C.c_void_p
        L.or_demod_free.argtypes = [C.c_void_p]
        L.or_demod_demodulate.argtypes = [C.c_void_p, _f32p, C.c_long, C.c_char_p, C.c_long]
        L.or_demod_demodulate.restype = C.c_long
        L.or_demod_demodulate_ex.argtypes = [C.c_void_p, _f32p, C.c_long, C.c_char_p, C.c_long,
                                             _f32p, C.c_long, _i64p, _i64p]
        L.or_demod_demodulate_ex.restype = C.c_long
        L.or_demod_constellation.argtypes = [C.c_void_p, _f32p, C.c_long, _f32p, C.c_long]
        L.or_demod_constellation.restype = C.c_long
        L.or_demod_bytes.argtypes = [C.c_void_p, _f32p, C.c_long, _u8p, C.c_int, _u8p, C.c_int,
                                     _u8p, C.c_long]
        L.or_demod_bytes.restype = C.c_long
        L.or_demod_gains.argtypes = [C.c_void_p] + [_f64p] * 5
        L.or_demod_rrc_f32.argtypes = [C.c_void_p, _f32p, C.c_int]
        L.or_demod_rrc_f32.restype = C.c_int
        L.or_bits_to_bytes.argtypes = [C.c_char_p, C.c_long, C.c_int, _u8p, C.c_long]
        L.or_bits_to_bytes.restype = C.c_long
        L.or_index_of.argtypes = [_u8p, C.c_long, _u8p, C.c_long]
        L.or_index_of.restype = C.c_long
        L.or_demod_batch.argtypes = [C.POINTER(DemodCfg), C.c_int, _f32p, C.c_long, C.c_long,
                                     C.c_char_p, C.c_long, _i64p, C.c_int]
        L.or_demod_batch.restype = C.c_int
        L.or_demod_batch_packed.argtypes = [C.POINTER(DemodCfg), C.c_int, _f32p, C.c_long, C.c_long,
                                            C.c_void_p, C.c_long, C.c_void_p, C.c_void_p, C.c_long,
                                            C.c_void_p, C.c_int]
        L.or_demod_batch_packed.restype = C.c_int
        L.or_modulate.argtypes = [C.c_int, C.c_int, C.c_double, C.c_int, C.c_int, C.c_char_p,
                                  C.c_char_p, C.c_long, C.c_int, _f32p, C.c_long]
        L.or_modulate.restype = C.c_long
        L.or_nco_new.argtypes = [C.c_double, C.c_double, C.c_double, C.c_double, C.c_uint64]
        L.or_nco_new.restype = C.c_void_p
        L.or_nco_free.argtypes = [C.c_void_p]
        L.or_nco_next.argtypes = [C.c_void_p, _f64p, _f64p]
        L.or_apply_lo_pair.argtypes = [C.c_void_p, C.c_void_p, _f32p, C.c_long]
        L.or_iqb_process.argtypes = [C.POINTER(IQB), _f32p, _f32p, C.c_long, C.c_int]
        L.or_sincos_batch.argtypes = [_f64p, C.c_long, _f64p, _f64p]
        _lib = L
    return _lib


def _fp(a):
    return a.ctypes.data_as(_f32p)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def rrc_taps(span, beta, fs, rs):
    out = np.zeros(4096, dtype=np.float64)
    n = lib().or_rrc_taps(float(span), float(beta), int(fs), int(rs), out.ctypes.data_as(_f64p), 4096)
    if n <= 0:
        raise ValueError("bad RRC parameters")
    return out[:n].copy()


def oracle_fir(taps_iq, x_iq, lanes=8):
    """One streaming ComplexFIRFilter over x (interleaved float32)."""
    taps_iq = _f32(taps_iq)
    x_iq = _f32(x_iq)
    h = lib().or_cfir_new(_fp(taps_iq), taps_iq.size, lanes)
    y = np.zeros_like(x_iq)
    lib().or_cfir_filter(h, _fp(x_iq), _fp(y), x_iq.size // 2)
    lib().or_cfir_free(h)
    return y


class OracleMM:
    def __init__(self, sps, kp, ki):
        self._h = lib().or_mm_new(sps, kp, ki)

    def process(self, x_iq, out_floats=None):
        x_iq = _f32(x_iq)
        cap = x_iq.size if out_floats is None else out_floats
        out = np.zeros(max(cap, 2), dtype=np.float32)
        n = lib().or_mm_process(self._h, _fp(x_iq), x_iq.size, _fp(out), cap)
        return out[: 2 * n].copy()

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_mm_free(self._h)


class OracleCostas:
    def __init__(self, fs, bw_hz, damping=0.707, trig=TRIG_PORTABLE):
        self._h = lib().or_costas_new(fs, bw_hz, damping, trig)

    def process(self, syms_iq):
        syms_iq = _f32(syms_iq)
        out = np.zeros_like(syms_iq)
        oi, oq = C.c_float(), C.c_float()
        L = lib()
        for k in range(syms_iq.size // 2):
            L.or_costas_process(self._h, float(syms_iq[2 * k]), float(syms_iq[2 * k + 1]),
                                C.byref(oi), C.byref(oq))
            out[2 * k] = oi.value
            out[2 * k + 1] = oq.value
        return out

    def state(self):
        t, f = C.c_double(), C.c_double()
        lib().or_costas_state(self._h, C.byref(t), C.byref(f))
        return t.value, f.value

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_costas_free(self._h)


class OracleFLL:
    def __init__(self, sps, rolloff, filter_size, bandwidth, lanes=8, trig=TRIG_PORTABLE):
        self._h = lib().or_fll_new(sps, rolloff, filter_size, bandwidth, lanes, trig)
        if not self._h:
            raise ValueError("ArgumentOutOfRangeException (Band-Edge Filter.cs:42-45)")
        self.filter_size = filter_size

    def process(self, x_iq):
        x_iq = _f32(x_iq)
        y = np.zeros_like(x_iq)
        lib().or_fll_process(self._h, _fp(x_iq), _fp(y), x_iq.size // 2)
        return y

    def taps(self):
        lo = np.zeros(2 * self.filter_size, dtype=np.float32)
        up = np.zeros_like(lo)
        lib().or_fll_taps(self._h, _fp(lo), _fp(up), lo.size)
        return lo, up

    def state(self):
        p, f = C.c_float(), C.c_float()
        lib().or_fll_state(self._h, C.byref(p), C.byref(f))
        return p.value, f.value

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_fll_free(self._h)


def demod_cfg(sample_rate, symbol_rate, rrc_alpha=0.9, rrc_span=6, symbol_sync_bw=0.0001,
              costas_loop_bw=120.0, cfo_loop_bw=None, differential=True, tsc=None,
              enable_fll=False, lanes=8, trig=TRIG_PORTABLE, ring_capacity=300_000_000,
              iq_balance=False):
    c = DemodCfg()
    lib().or_demod_cfg_default(C.byref(c), int(sample_rate), int(symbol_rate))
    c.rrc_alpha = float(np.float32(rrc_alpha))
    c.rrc_span = int(rrc_span)
    c.symbol_sync_bw = float(symbol_sync_bw)
    c.costas_loop_bw = float(costas_loop_bw)
    if cfo_loop_bw is not None:
        c.cfo_loop_bw = float(cfo_loop_bw)
    c.differential = 1 if differential else 0
    c.tsc = tsc.encode() if tsc else None
    c.enable_fll = 1 if enable_fll else 0
    c.lanes = int(lanes)
    c.trig_mode = int(trig)
    c.ring_capacity = int(ring_capacity)
    c.iq_balance = 1 if iq_balance else 0
    return c


ERR_INDEX = -3   # OR_ERR_INDEX


def _raise(n):
    """The C# exception a negative oracle return stands for."""
    if n == -1:
        raise ValueError("Samples must be interleaved IQ with even length.")
    if n == ERR_INDEX:
        raise IndexError("IndexOutOfRangeException: NaN symbol timing pinned baseIndex at 0 "
                         "(MuellerMuller.cs:113-115, 164)")


class OracleIQBalancer:
    """IQ_Balancer (IQ Balancer.cs:10-26); literal=True keeps the reference's
    loop bound (the first half of the complex samples, the rest of OUT left as
    it was: zeros here)."""

    def __init__(self):
        self._st = IQB(0.0, 0.0)

    def process(self, x_iq, literal=False):
        x = _f32(x_iq)
        y = np.zeros_like(x)
        lib().or_iqb_process(C.byref(self._st), _fp(x), _fp(y), x.size, 1 if literal else 0)
        return y


class OracleDemod:
    """QPSKDeModulator restated (QPSKDeModulator.cs:11-457)."""

    def __init__(self, sample_rate, symbol_rate, rrc_alpha=0.9, rrc_span=6, symbol_sync_bw=0.0001,
                 costas_loop_bw=120.0, cfo_loop_bw=None, differential=True, tsc=None,
                 enable_fll=False, lanes=8, trig=TRIG_PORTABLE, ring_capacity=300_000_000,
                 iq_balance=False):
        self._cfg = demod_cfg(sample_rate, symbol_rate, rrc_alpha, rrc_span, symbol_sync_bw,
                              costas_loop_bw, cfo_loop_bw, differential, tsc, enable_fll, lanes,
                              trig, ring_capacity, iq_balance)
        self._tsc_keep = self._cfg.tsc
        err = C.c_int()
        self._h = lib().or_demod_new(C.byref(self._cfg), C.byref(err))
        if not self._h:
            if err.value == 1:
                raise ValueError("ArgumentOutOfRangeException (Band-Edge Filter.cs:42-45)")
            raise ValueError("invalid demodulator parameters")

    def DeModulate(self, iq) -> str:
        iq = _f32(iq)
        cap = iq.size + 16
        buf = C.create_string_buffer(cap)
        n = lib().or_demod_demodulate(self._h, _fp(iq), iq.size, buf, cap)
        _raise(n)
        return buf.raw[:n].decode()

    def demodulate_ex(self, iq):
        """Raw bits (before TSC strip), rotated symbols and the TSC start index."""
        iq = _f32(iq)
        cap = iq.size + 16
        buf = C.create_string_buffer(cap)
        syms = np.zeros(max(iq.size, 2), dtype=np.float32)
        ns, ti = C.c_long(), C.c_long()
        n = lib().or_demod_demodulate_ex(self._h, _fp(iq), iq.size, buf, cap, _fp(syms), syms.size,
                                         C.byref(ns), C.byref(ti))
        _raise(n)
        return buf.raw[:n].decode(), syms[: 2 * ns.value].copy(), ti.value

    def deModulateConstellation(self, iq):
        iq = _f32(iq)
        out = np.zeros(max(iq.size, 2), dtype=np.float32)
        n = lib().or_demod_constellation(self._h, _fp(iq), iq.size, _fp(out), out.size)
        _raise(n)
        return out[: 2 * n].copy()

    def DeModulateBytes(self, iq, start: bytes, end: bytes) -> bytes:
        iq = _f32(iq)
        if len(start) == 0:
            raise ValueError("startMarker cannot be empty.")
        if len(end) == 0:
            raise ValueError("endMarker cannot be empty.")
        s = np.frombuffer(start, dtype=np.uint8).copy()
        e = np.frombuffer(end, dtype=np.uint8).copy()
        cap = iq.size // 8 + 16
        out = np.zeros(cap, dtype=np.uint8)
        n = lib().or_demod_bytes(self._h, _fp(iq), iq.size, s.ctypes.data_as(_u8p), s.size,
                                 e.ctypes.data_as(_u8p), e.size, out.ctypes.data_as(_u8p), cap)
        _raise(n)
        return bytes(out[:n])

    def DeModulateTextUtf8(self, iq, start="\u0002", end="\u0003") -> str:
        p = self.DeModulateBytes(iq, start.encode("utf-8"), end.encode("utf-8"))
        return p.decode("utf-8", errors="replace") if p else ""

    def gains(self):
        v = [C.c_double() for _ in range(5)]
        lib().or_demod_gains(self._h, *[C.byref(x) for x in v])
        return dict(zip(["mm_sps", "kp", "ki", "costas_alpha", "costas_beta"], [x.value for x in v]))

    def rrc_f32(self):
        out = np.zeros(4096, dtype=np.float32)
        n = lib().or_demod_rrc_f32(self._h, _fp(out), 4096)
        return out[:n].copy()

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_demod_free(self._h)


def demod_batch(iq2d, sample_rate, symbol_rate, n_threads=1, **kw):
    """S independent reference demodulators over rows of iq2d ([S, 2n] float32).
    Returns (list of bit strings)."""
    iq2d = np.ascontiguousarray(iq2d, dtype=np.float32)
    S, nf = iq2d.shape
    cfg = demod_cfg(sample_rate, symbol_rate, **kw)
    cap = nf + 16
    bits = C.create_string_buffer(S * cap)
    nb = np.zeros(S, dtype=np.int64)
    rc = lib().or_demod_batch(C.byref(cfg), S, _fp(iq2d), nf, nf, bits, cap,
                              nb.ctypes.data_as(_i64p), int(n_threads))
    if rc:
        raise ValueError("oracle batch failed %d" % rc)
    raw = bits.raw
    return [raw[s * cap: s * cap + int(nb[s])].decode() for s in range(S)]


def demod_batch_timed(iq2d, sample_rate, symbol_rate, n_threads=1, **kw):
    """Same as demod_batch but returns only bit counts (for timing)."""
    iq2d = np.ascontiguousarray(iq2d, dtype=np.float32)
    S, nf = iq2d.shape
    cfg = demod_cfg(sample_rate, symbol_rate, **kw)
    nb = np.zeros(S, dtype=np.int64)
    rc = lib().or_demod_batch(C.byref(cfg), S, _fp(iq2d), nf, nf, None, 0,
                              nb.ctypes.data_as(_i64p), int(n_threads))
    if rc:
        raise ValueError("oracle batch failed %d" % rc)
    return nb


def demod_batch_packed(iq2d, sample_rate, symbol_rate, n_threads=1, want_bits=True,
                       want_syms=False, **kw):
    """One DeModulate call per row of iq2d ([S, 2n] float32) on n_threads host
    threads.  Returns (bits [S, B] uint8 packed MSB-first like the GPU rows or
    None, n_bits [S], syms [S, 2n] float32 or None, n_syms [S])."""
    iq2d = np.ascontiguousarray(iq2d, dtype=np.float32)
    S, nf = iq2d.shape
    cfg = demod_cfg(sample_rate, symbol_rate, **kw)
    bstride = (nf + 7) // 8 + 8
    bits = np.zeros((S, bstride), dtype=np.uint8) if want_bits else None
    syms = np.zeros((S, max(nf, 2)), dtype=np.float32) if want_syms else None
    nb = np.zeros(S, dtype=np.int64)
    ns = np.zeros(S, dtype=np.int64)
    rc = lib().or_demod_batch_packed(C.byref(cfg), S, _fp(iq2d), nf, nf,
                                     bits.ctypes.data if bits is not None else None, bstride,
                                     nb.ctypes.data, syms.ctypes.data if syms is not None else None,
                                     syms.shape[1] if syms is not None else 0, ns.ctypes.data,
                                     int(n_threads))
    if rc:
        raise ValueError("oracle batch failed %d" % rc)
    return bits, nb, syms, ns


def modulate(sample_rate, symbol_rate, bits: str, rrc_alpha=0.9, rrc_span=6, differential=True,
             tsc=None, pulse_shaping=True):
    """QPSKModulator.Modulate restated (FFT filter replaced by direct convolution)."""
    total_bits = len(bits) + (len(tsc) if tsc else 0)
    cap = 2 * ((total_bits // 2) * max(1, sample_rate // symbol_rate) + 8192) + 16
    out = np.zeros(cap, dtype=np.float32)
    n = lib().or_modulate(int(sample_rate), int(symbol_rate), float(rrc_alpha), int(rrc_span),
                          1 if differential else 0, tsc.encode() if tsc else None, bits.encode(),
                          len(bits), 1 if pulse_shaping else 0, _fp(out), cap)
    if n < 0:
        raise ValueError("modulate failed")
    return out[:n].copy()


def bytes_to_bits(data: bytes) -> str:
    """BitPacker.BytesToBitString (HelperFunctions.cs:14-29), MSB first."""
    return "".join(format(b, "08b") for b in data)


def modulate_bytes(sample_rate, symbol_rate, payload: bytes, start: bytes, end: bytes, **kw):
    """QPSKModulator.ModulateBytes (QPSKModulator.cs:54-72)."""
    return modulate(sample_rate, symbol_rate, bytes_to_bits(start + payload + end), **kw)


def modulate_text_utf8(sample_rate, symbol_rate, text, start="\u0002", end="\u0003", **kw):
    return modulate_bytes(sample_rate, symbol_rate, text.encode("utf-8"), start.encode("utf-8"),
                          end.encode("utf-8"), **kw)


class OracleNCO:
    def __init__(self, freq_hz, fs, ppm=0.0, phase0=0.0, seed=1):
        self._h = lib().or_nco_new(freq_hz, fs, ppm, phase0, seed)

    def next(self):
        r, i = C.c_double(), C.c_double()
        lib().or_nco_next(self._h, C.byref(r), C.byref(i))
        return complex(r.value, i.value)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_nco_free(self._h)


def apply_lo_pair(tx: OracleNCO, rx: OracleNCO, iq):
    """testAtDataLevel.cs:39-42 channel: iq *= tx.Next() * conj(rx.Next())."""
    iq = _f32(iq).copy()
    lib().or_apply_lo_pair(tx._h, rx._h, _fp(iq), iq.size // 2)
    return iq


def sincos(x):
    """Portable sincos of the oracle (or_sincos.h) over a float64 array."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    s = np.zeros_like(x)
    c = np.zeros_like(x)
    lib().or_sincos_batch(x.ctypes.data_as(_f64p), x.size, s.ctypes.data_as(_f64p),
                          c.ctypes.data_as(_f64p))
    return s, c
