"""Independent numpy / pure-Python restatement of the reference chain.

Second, independent reading of the C# (written separately from
oracle/qpsk_oracle.c) used only to cross-check the C oracle on small inputs.
Float ops use numpy float32 scalars/arrays (IEEE single, one rounding per op),
double ops use Python floats; no op is fused.

References: FIRFilter.cs:144-211, MuellerMuller.cs:52-190,
CostasLoopQpsk.cs:29-92, QPSKDeModulator.cs:39-56,304-408, RRC-filter.cs:16-75.
"""
from __future__ import annotations

import math
from fractions import Fraction

import numpy as np

F = np.float32


def rrc_taps(span, beta, fs, rs):
    """RRC-filter.cs:16-75 (double)."""
    sps = int(round(fs / rs))  # Python round() is half-even like Math.Round
    span_i = int(round(span))
    taps = span_i * sps + 1
    mid = (taps - 1) // 2
    h = []
    for n in range(taps):
        t = (n - mid) / float(sps)
        if abs(t) < 1e-8:
            v = 1.0 + beta * (4.0 / math.pi - 1.0)
        elif abs(abs(t) - 1.0 / (4.0 * beta)) < 1e-8:
            v = (beta / math.sqrt(2.0)) * ((1.0 + 2.0 / math.pi) * math.sin(math.pi / (4.0 * beta))
                                           + (1.0 - 2.0 / math.pi) * math.cos(math.pi / (4.0 * beta)))
        else:
            num = math.sin(math.pi * t * (1.0 - beta)) + 4.0 * beta * t * math.cos(math.pi * t * (1.0 + beta))
            den = math.pi * t * (1.0 - math.pow(4.0 * beta * t, 2.0))
            v = num / den
        h.append(v)
    e = 0.0
    for v in h:
        e += v * v
    nrm = math.sqrt(e)
    return np.array([v / nrm for v in h], dtype=np.float64)


def fir_real_taps(h_f32, x_iq, lanes=8):
    """ComplexFIRFilter.Filter over a whole buffer with imag taps = 0,
    vectorised over output index; per-output summation order of the C#
    Vector<float> path (FIRFilter.cs:156-192)."""
    h = np.asarray(h_f32, dtype=F)
    T = h.size
    x = np.asarray(x_iq, dtype=F).reshape(-1, 2)
    n = x.shape[0]
    xp = np.concatenate([np.zeros((T - 1, 2), F), x])
    hrev = h[::-1].copy()
    zero = F(0)
    out = np.zeros((n, 2), F)
    for comp in range(2):
        other = 1 - comp
        win = lambda k, c: xp[k:k + n, c]
        def term(k):
            # (hi*xi) - (hq*xq) for I ; (hi*xq) + (hq*xi) for Q, hq = 0
            if comp == 0:
                return (hrev[k] * win(k, 0)) - (zero * win(k, 1))
            return (hrev[k] * win(k, 1)) + (zero * win(k, 0))
        acc = np.zeros(n, F)
        if lanes > 1:
            nvec = T - T % lanes
            for l in range(lanes):
                a = np.zeros(n, F)
                for i in range(0, nvec, lanes):
                    a = a + term(i + l)
                acc = acc + a
            for k in range(nvec, T):
                acc = acc + term(k)
        else:
            for k in range(T):
                acc = acc + term(k)
        out[:, comp] = acc
    return out.reshape(-1)


def mm_gains(bn):
    zeta = 1.0 / math.sqrt(2.0)
    wn = ((2.0 * math.pi * bn) / (zeta + 0.25) / zeta)
    den = 1.0 + 2.0 * zeta * wn + wn * wn
    return (4.0 * zeta * wn) / den, (4.0 * wn * wn) / den


class MM:
    """MuellerMuller.cs (single-call semantics incl. buffer carry)."""

    def __init__(self, sps, kp, ki):
        self.sps, self.kp, self.ki = sps, kp, ki
        self.base, self.mu, self.integ = 1, 0.0, 0.0
        self.ps = (F(0), F(0))
        self.pd = (F(0), F(0))
        self.has_prev = False
        self.buf = np.zeros((0, 2), F)

    def process(self, x_iq, out_floats=None):
        x = np.asarray(x_iq, dtype=F).reshape(-1, 2)
        cap = x.size if out_floats is None else out_floats
        self.buf = np.concatenate([self.buf, x])
        cnt = self.buf.shape[0]
        out = []
        while self.base + 2 < cnt:
            b = self.buf[self.base - 1:self.base + 3]
            t = F(self.mu)
            tm1, tm2, tp1 = t - F(1), t - F(2), t + F(1)
            cm1 = -(t * tm1 * tm2) * (F(1) / F(6))
            c0 = (tp1 * tm1 * tm2) * (F(1) / F(2))
            c1 = -(tp1 * t * tm2) * (F(1) / F(2))
            c2 = (tp1 * t * tm1) * (F(1) / F(6))
            ci = cm1 * b[0, 0] + c0 * b[1, 0] + c1 * b[2, 0] + c2 * b[3, 0]
            cq = cm1 * b[0, 1] + c0 * b[1, 1] + c1 * b[2, 1] + c2 * b[3, 1]
            di = F(1) if ci >= 0 else F(-1)
            dq = F(1) if cq >= 0 else F(-1)
            if self.has_prev:
                t1 = float(self.pd[0]) * float(ci) + float(self.pd[1]) * float(cq)
                t2 = float(di) * float(self.ps[0]) + float(dq) * float(self.ps[1])
                e = t1 - t2
                self.integ += self.ki * e
                corr = self.kp * e + self.integ
                corr = min(corr, 0.1) if corr > 0.1 else corr
                corr = -0.1 if corr < -0.1 else corr
                adv = self.sps + corr
            else:
                self.has_prev = True
                adv = self.sps
            if 2 * len(out) + 1 >= cap:
                break
            out.append((ci, cq))
            self.ps, self.pd = (ci, cq), (di, dq)
            nt = (float(self.base) + self.mu) + adv
            self.base = int(math.floor(nt))
            self.mu = nt - float(self.base)
            if self.base + 1 >= cnt:
                break
        consumed = min(max(0, self.base - 1), max(0, cnt - 3))
        if consumed > 0:
            self.buf = self.buf[consumed:]
            self.base -= consumed
        return np.array(out, dtype=F).reshape(-1)


# ---- portable sincos (exact-fma emulation of or_sincos.h / qpsk_sincos.h) ----
def _fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))


# The table is recomputed here independently of tools/gen_sincos_table.py
# (different pi source and series grouping): sin/cos(k pi/256) as a correctly
# rounded double head plus the tail rounded to float.
_PI_DIGITS = "3.14159265358979323846264338327950288419716939937510582097494459230781640628620899"


def _table():
    from decimal import Decimal, localcontext
    out = []
    with localcontext() as ctx:
        ctx.prec = 70
        pi = Decimal(_PI_DIGITS)
        for k in range(512):
            a = pi * k / 256
            # sin and cos from one pass over the exp series terms a^n/n!
            term, sn, cs, n = Decimal(1), Decimal(0), Decimal(0), 0
            while n < 90:
                cs += term if n % 4 == 0 else (-term if n % 4 == 2 else 0)
                sn += term if n % 4 == 1 else (-term if n % 4 == 3 else 0)
                n += 1
                term = term * a / n
            row = []
            for v in (sn, cs):
                if abs(v) < Decimal("1e-40"):
                    row += [0.0, 0.0]
                else:
                    hi = float(v)
                    row += [hi, float(np.float32(float(v - Decimal(hi))))]
            out.append(tuple(row))
    return out


SINCOS_TABLE = _table()


def portable_sincos(x):
    if not (abs(x) <= 2.0 ** 40):   # huge, +-Inf (-> NaN) and NaN
        if math.isnan(x) or math.isinf(x):
            return math.nan, math.nan
        x = math.fmod(x, 6.28318530717958647693)
    sh = float.fromhex("0x1.8p+52")
    k = _fma(x, float.fromhex("0x1.45f306dc9c883p+6"), sh) - sh   # rint of the exact product
    r = _fma(-k, float.fromhex("0x1.921fb54442d18p-7"), x)
    r = _fma(-k, float.fromhex("0x1.1a62633145c07p-61"), r)
    ts, ls, tc, lc = SINCOS_TABLE[int(k) & 511]
    z = r * r
    r3p = (r * z) * _fma(z, 1.0 / 120.0, -1.0 / 6.0)
    cm = z * _fma(z, _fma(z, -1.0 / 720.0, 1.0 / 24.0), -0.5)
    return (ts + _fma(tc, r, _fma(tc, r3p, _fma(ts, cm, ls))),
            tc + _fma(-ts, r, _fma(-ts, r3p, _fma(tc, cm, lc))))


class Costas:
    """CostasLoopQpsk.cs:29-92."""

    def __init__(self, fs, bw_hz, damping=0.707, portable=True):
        bw = 2.0 * math.pi * bw_hz / fs
        d = 1.0 + 2.0 * damping * bw + bw * bw
        self.alpha = (4.0 * damping * bw) / d
        self.beta = (4.0 * bw * bw) / d
        self.theta = 0.0
        self.freq = 0.0
        self.portable = portable

    def process(self, i, q):
        if self.portable:
            s, c = portable_sincos(self.theta)
        else:
            c, s = math.cos(self.theta), math.sin(self.theta)
        mi = float(i) * c + float(q) * s
        mq = float(q) * c - float(i) * s
        oi, oq = F(mi), F(mq)
        ei = 1.0 if oi >= 0 else -1.0
        eq = 1.0 if oq >= 0 else -1.0
        pe = ei * mq - eq * mi
        self.freq += self.beta * pe
        self.theta += self.freq + self.alpha * pe
        if self.theta > math.pi:
            self.theta -= 2.0 * math.pi
        elif self.theta < -math.pi:
            self.theta += 2.0 * math.pi
        return oi, oq


def decode_bits(rot, differential=True, state=None):
    """QPSKDeModulator.cs:372-408 + AppendDeltaBits/AppendDecisionBits."""
    st = state if state is not None else {"have": False, "p": (F(0), F(0))}
    out = []
    for ri, rq in rot:
        di = F(1) if ri >= 0 else F(-1)
        dq = F(1) if rq >= 0 else F(-1)
        if differential:
            if not st["have"]:
                st["p"] = (di, dq)
                st["have"] = True
                continue
            pi_, pq = st["p"]
            dli = di * pi_ + dq * pq
            dlq = dq * pi_ - di * pq
            st["p"] = (di, dq)
            if abs(dli) >= abs(dlq):
                out.append("00" if dli >= 0 else "11")
            else:
                out.append("01" if dlq >= 0 else "10")
        else:
            if di < 0:
                out.append("00" if dq < 0 else "01")
            else:
                out.append("11" if dq >= 0 else "10")
    return "".join(out), st


class RefDemod:
    """QPSKDeModulator.DeModulate (FLL off), independent model."""

    def __init__(self, fs, rs, alpha, span, ssbw=1e-4, clbw=120.0, differential=True, lanes=8,
                 portable=True):
        self.h = rrc_taps(float(span), float(F(alpha)), fs, rs).astype(F)
        kp, ki = mm_gains(ssbw)
        self.mm = MM(fs / float(rs), kp, ki)
        self.costas = Costas(float(rs), rs / clbw, 0.707, portable)
        self.lanes = lanes
        self.hist = np.zeros(2 * (self.h.size - 1), F)
        self.diff = {"have": False, "p": (F(0), F(0))}
        self.differential = differential

    def demodulate(self, iq):
        iq = np.asarray(iq, dtype=F)
        xx = np.concatenate([self.hist, iq])
        y = fir_real_taps(self.h, xx, self.lanes)[self.hist.size:]
        self.hist = xx[-self.hist.size:] if self.hist.size else self.hist
        syms = self.mm.process(y, iq.size).reshape(-1, 2)
        rot = [self.costas.process(s[0], s[1]) for s in syms]
        bits, self.diff = decode_bits(rot, self.differential, self.diff)
        return bits, np.array(rot, dtype=F).reshape(-1), y


# ---- Band-Edge FLL (Band-Edge Filter.cs:40-202), independent model ----------
import ctypes as _ct

_libm = _ct.CDLL("libm.so.6")
_libm.sinf.argtypes = [_ct.c_float]
_libm.sinf.restype = _ct.c_float
_libm.cosf.argtypes = [_ct.c_float]
_libm.cosf.restype = _ct.c_float
_libm.remainderf.argtypes = [_ct.c_float, _ct.c_float]
_libm.remainderf.restype = _ct.c_float
PI_F = F(3.14159274101257324219)


def _sinc(x):
    if x == F(0):
        return F(1)
    arg = PI_F * x
    return F(_libm.sinf(float(arg))) / arg


def fll_taps(sps, rolloff, n):
    sps, rolloff = F(sps), F(rolloff)
    mid = (n - 1) // 2
    bb = []
    s = F(0)
    for i in range(n):
        k = F(i - mid) / (F(2) * sps)
        pos = rolloff * k
        tap = _sinc(pos - F(0.5)) + _sinc(pos + F(0.5))
        s = s + tap
        bb.append(tap)
    bb = [b / s for b in bb]
    two_pi = F(2) * PI_F
    lo, up = [], []
    for i in range(n):
        k = F(i - mid) / (F(2) * sps)
        ang = -two_pi * (F(1) + rolloff) * k
        wc, ws = F(_libm.cosf(float(ang))), F(_libm.sinf(float(ang)))
        li, lq = bb[i] * wc, bb[i] * ws
        lo += [li, lq]
        up += [li, -lq]
    return np.array(lo, F), np.array(up, F)


class FLL:
    def __init__(self, sps, rolloff, n, bw, lanes=8):
        self.lo, self.up = fll_taps(sps, rolloff, n)
        self.n = n
        self.lanes = lanes
        sps = F(sps)
        self.beta = F(4) * F(bw) / sps
        self.alpha = F(0)
        self.maxf = (F(2) * PI_F) * (F(2) / sps)
        self.phase = F(0)
        self.freq = F(0)
        self.hist = [(F(0), F(0))] * n    # last n mixed samples, oldest first

    def _dot(self, taps, win):
        n, w = self.n, self.lanes
        hr = [(taps[2 * (n - 1 - k)], taps[2 * (n - 1 - k) + 1]) for k in range(n)]
        ai = aq = F(0)
        if w > 1:
            nvec = n - n % w
            vi = [F(0)] * w
            vq = [F(0)] * w
            for i in range(0, nvec, w):
                for l in range(w):
                    (hi, hq), (xi, xq) = hr[i + l], win[i + l]
                    vi[l] = vi[l] + ((hi * xi) - (hq * xq))
                    vq[l] = vq[l] + ((hi * xq) + (hq * xi))
            for l in range(w):
                ai = ai + vi[l]
                aq = aq + vq[l]
            rng = range(nvec, n)
        else:
            rng = range(n)
        for i in rng:
            (hi, hq), (xi, xq) = hr[i], win[i]
            ai = ai + ((hi * xi) - (hq * xq))
            aq = aq + ((hi * xq) + (hq * xi))
        return ai, aq

    def process(self, x_iq):
        x = np.asarray(x_iq, F).reshape(-1, 2)
        out = np.zeros_like(x)
        two_pi = F(2) * PI_F
        for t in range(x.shape[0]):
            # MathF.Sin / MathF.Cos (Band-Edge Filter.cs:108-109): the C runtime's
            c = F(_libm.cosf(float(self.phase)))
            s = F(_libm.sinf(float(self.phase)))
            xi, xq = x[t, 0], x[t, 1]
            oi = xi * c - xq * s
            oq = xi * s + xq * c
            out[t] = (oi, oq)
            self.hist = self.hist[1:] + [(oi, oq)]
            ui, uq = self._dot(self.up, self.hist)
            li, lq = self._dot(self.lo, self.hist)
            err = (li * li + lq * lq) - (ui * ui + uq * uq)
            self.freq = self.freq + self.beta * err
            self.phase = self.phase + (self.freq + self.alpha * err)
            if self.phase > two_pi or self.phase < -two_pi:
                self.phase = F(_libm.remainderf(float(self.phase), float(two_pi)))
            if self.freq > self.maxf:
                self.freq = self.maxf
            elif self.freq < -self.maxf:
                self.freq = -self.maxf
        return out.reshape(-1)


# ---------------------------------------------------------------------------
# Byte framer, on '0'/'1' strings exactly as the C# walks them
# (QPSKDeModulator.cs:57-259, HelperFunctions.cs:32-70).

def bits_to_bytes(bits: str, off: int) -> bytes:
    """BitPacker.BitsToBytes: MSB-first from bit `off`, trailing partial byte dropped."""
    n = (len(bits) - off) // 8
    if len(bits) - off < 8:
        return b""
    return int(bits[off:off + 8 * n], 2).to_bytes(n, "big")


class RefFramer:
    """One reference instance's framer fields and DeModulateBytes step, fed the
    post-TSC bit string of each call (rxBits, :178)."""

    def __init__(self, ring_capacity=300_000_000):
        self.cap = ring_capacity
        self.reset()

    def reset(self):                       # ResetFramer (:159-167)
        self.in_frame = False
        self.locked = -1
        self.carry = ""
        self.ring = bytearray()
        self.pack_byte = 0
        self.pack_bits = 0

    def _append(self, bits: str) -> int:   # AppendBitsToRing (:108-129)
        produced = 0
        for c in bits:
            self.pack_byte = ((self.pack_byte << 1) | (c == "1")) & 0xFF
            self.pack_bits += 1
            if self.pack_bits == 8:
                if len(self.ring) >= self.cap:
                    return -1
                self.ring.append(self.pack_byte)
                produced += 1
                self.pack_bits = 0
                self.pack_byte = 0
        return produced

    def _finish(self, appended: int, end: bytes) -> bytes:
        frm = max(0, len(self.ring) - (appended + len(end)))
        at = bytes(self.ring).find(end, frm)       # RingIndexOf (:133-149)
        if at >= 0:
            out = bytes(self.ring[:at])
            self.reset()
            return out
        return b""

    def push(self, rx: str, start: bytes, end: bytes) -> bytes:
        if not rx:
            return b""                              # :179-180
        if not self.in_frame:
            cand = self.carry + rx
            for off in range(8):                    # :187-230
                by = bits_to_bytes(cand, off)
                s = by.find(start)
                if not by or s < 0:
                    continue
                mend = off + 8 * (s + len(start))
                if mend > len(cand):
                    continue
                self.in_frame = True
                self.locked = off
                self.ring = bytearray()
                self.pack_byte = self.pack_bits = 0
                appended = self._append(cand[mend:])
                if appended < 0:
                    self.reset()
                    return b""
                return self._finish(appended, end)
            keep = min(len(cand), len(start) * 8 + 7)   # :233-235
            self.carry = cand[len(cand) - keep:] if keep else ""
            return b""
        appended = self._append(rx)
        if appended < 0:
            self.reset()
            return b""
        return self._finish(appended, end)
