/*
 * qpsk_glibc_trig.h -- PRODUCT restatement of glibc's double sin and cos, the
 * functions .NET's Math.Sin / Math.Cos call on a Linux x86-64 host (the Costas
 * loop's NCO, CostasLoopQpsk.cs:69-70), for qpsk_demod_params.costas_trig = 1.
 *
 * glibc 2.35 sysdeps/ieee754/dbl-64/s_sin.c as its x86-64 FMA ifunc variant
 * evaluates it (every a*b +- c gcc contracts is an explicit fma here), with
 * the generic __branred (branred.c, no fma) for |x| >= 105414350.  The oracle
 * keeps its own copy (oracle/or_glibc_trig.h); tools/check_glibc_sin.c checks
 * the oracle copy against the real libm (680M inputs: 0 differences) and
 * tests/test_oracle.py checks this copy against the oracle's.
 *
 * Host + device.  The sincos table is passed in (the loop kernel stages it in
 * LDS); toverp (Payne-Hanek, rare) is read from the constant copy.  Compile
 * with -ffp-contract=off (the fma calls are explicit).
 *
 * Licence: this restates the algorithm and constants of glibc's s_sin.c and
 * branred.c (Copyright (C) 2001-2022 Free Software Foundation, Inc., IBM
 * Accurate Mathematical Library), which are LGPL-2.1-or-later; this file and
 * qpsk_glibc_tables.h carry that code's terms.  Pinned to glibc 2.35, x86-64
 * FMA variant (tests/test_oracle.py GLIBC_PIN).
 */
#ifndef QPSK_GLIBC_TRIG_H
#define QPSK_GLIBC_TRIG_H
#include <math.h>
#include <stdint.h>

#include "qpsk_glibc_tables.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define QPSK_GHD __host__ __device__
#else
#define QPSK_GHD
#endif

static const double qpsk_gl_sincostab_host[440] = {QPSK_GLIBC_SINCOSTAB_VALUES};
#if defined(__HIPCC__)
static __device__ const double qpsk_gl_sincostab_dev[440] = {QPSK_GLIBC_SINCOSTAB_VALUES};
static __device__ const double qpsk_gl_toverp_dev[75] = {QPSK_GLIBC_TOVERP_VALUES};
#endif
static const double qpsk_gl_toverp_host[75] = {QPSK_GLIBC_TOVERP_VALUES};

QPSK_GHD static inline const double *qpsk_gl_toverp(void)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return qpsk_gl_toverp_dev;
#else
    return qpsk_gl_toverp_host;
#endif
}

QPSK_GHD static inline uint64_t qpsk_gl_bits(double x)
{
    union { double d; uint64_t u; } v;
    v.d = x;
    return v.u;
}

QPSK_GHD static inline double qpsk_gl_from_bits(uint64_t u)
{
    union { double d; uint64_t u; } v;
    v.u = u;
    return v.d;
}

/* usncs.h / s_sin.c constants */
#define QPSK_GL_S1 (-0x1.5555555555555p-3)
#define QPSK_GL_S2 (0x1.1111111110ecep-7)
#define QPSK_GL_S3 (-0x1.a01a019db08b8p-13)
#define QPSK_GL_S4 (0x1.71de27b9a7ed9p-19)
#define QPSK_GL_S5 (-0x1.addffc2fcdf59p-26)
#define QPSK_GL_SN3 (-0x1.5555555555515p-3)
#define QPSK_GL_SN5 (0x1.11110e829872fp-7)
#define QPSK_GL_CS2 (0x1p-1)
#define QPSK_GL_CS4 (-0x1.5555555555535p-5)
#define QPSK_GL_CS6 (0x1.6c16bedd9e239p-10)
#define QPSK_GL_BIG (0x1.8p45)
#define QPSK_GL_HP0 (0x1.921fb54442d18p0)
#define QPSK_GL_HP1 (0x1.1a62633145c07p-54)
#define QPSK_GL_MP1 (0x1.921fb58p0)
#define QPSK_GL_MP2 (-0x1.dde973cp-27)
#define QPSK_GL_PP3 (-0x1.cb3b398p-55)
#define QPSK_GL_PP4 (-0x1.d747f23e32ed7p-83)
#define QPSK_GL_HPINV (0x1.45f306dc9c883p-1)
#define QPSK_GL_TOINT (0x1.8p52)

/* TAYLOR_SIN (s_sin.c): a + ((POLY(xx) * a - 0.5 * da) * xx + da) */
QPSK_GHD static inline double qpsk_gl_taylor_sin(double a, double da)
{
    const double xx = a * a;
    double p = fma(xx, QPSK_GL_S5, QPSK_GL_S4);
    p = fma(xx, p, QPSK_GL_S3);
    p = fma(xx, p, QPSK_GL_S2);
    p = fma(xx, p, QPSK_GL_S1);
    const double t = fma(xx, fma(p, a, -(0.5 * da)), da);
    return a + t;
}

/* table index of u = big + |x|: its low word, times 4 */
QPSK_GHD static inline int qpsk_gl_tab_index(double u)
{
    return (int)((uint32_t)qpsk_gl_bits(u) << 2);
}

QPSK_GHD static inline double qpsk_gl_do_cos(double x, double dx, const double *tab)
{
    if (x < 0) dx = -dx;
    const double ax = fabs(x);
    const double u = QPSK_GL_BIG + ax;
    const double xr = (ax - (u - QPSK_GL_BIG)) + dx;
    const double xx = xr * xr;
    const double s = fma(xr * xx, fma(xx, QPSK_GL_SN5, QPSK_GL_SN3), xr);
    const double c = xx * fma(xx, fma(xx, QPSK_GL_CS6, QPSK_GL_CS4), QPSK_GL_CS2);
    const double *t = tab + qpsk_gl_tab_index(u);
    const double sn = t[0], ssn = t[1], cs = t[2], ccs = t[3];
    double cor = fma(-s, ssn, ccs);
    cor = fma(-c, cs, cor);
    cor = fma(-s, sn, cor);
    return cs + cor;
}

QPSK_GHD static inline double qpsk_gl_do_sin(double x, double dx, const double *tab)
{
    const double xold = x;
    if (fabs(x) < 0.126) return qpsk_gl_taylor_sin(x, dx);
    if (x <= 0) dx = -dx;
    const double ax = fabs(x);
    const double u = QPSK_GL_BIG + ax;
    const double xr = ax - (u - QPSK_GL_BIG);
    const double xx = xr * xr;
    const double s = xr + fma(xr * xx, fma(xx, QPSK_GL_SN5, QPSK_GL_SN3), dx);
    const double c = fma(xr, dx, xx * fma(xx, fma(xx, QPSK_GL_CS6, QPSK_GL_CS4), QPSK_GL_CS2));
    const double *t = tab + qpsk_gl_tab_index(u);
    const double sn = t[0], ssn = t[1], cs = t[2], ccs = t[3];
    double cor = fma(s, ccs, ssn);
    cor = fma(-c, sn, cor);
    cor = fma(s, cs, cor);
    return copysign(sn + cor, xold);
}

/* x = n pi/2 + (a + da), |x| < 105414350 (s_sin.c reduce_sincos) */
QPSK_GHD static inline int qpsk_gl_reduce_sincos(double x, double *a, double *da)
{
    const double t = fma(x, QPSK_GL_HPINV, QPSK_GL_TOINT);
    const double xn = t - QPSK_GL_TOINT;
    double y = fma(-xn, QPSK_GL_MP1, x);
    y = fma(-xn, QPSK_GL_MP2, y);
    const int n = (int)(qpsk_gl_bits(t) & 3);
    const double t2 = fma(-xn, QPSK_GL_PP3, y);
    double db = fma(-xn, QPSK_GL_PP3, y - t2);
    const double b = fma(-xn, QPSK_GL_PP4, t2);
    db = db + fma(-xn, QPSK_GL_PP4, t2 - b);
    *a = b;
    *da = db;
    return n;
}

/* branred.c: one of the two halves of x (x1 / x2) against 2/pi */
QPSK_GHD static inline void qpsk_gl_branred_part(double xi, double *bo, double *bbo, double *sumo)
{
    const double big = 0x1.8p52, big1 = 0x1.8p54;
    double r[6], s, t, sum = 0, b, bb;
    const double *toverp = qpsk_gl_toverp();
    int k = (int)((((int64_t)qpsk_gl_bits(xi)) >> 52) & 2047);
    k = (k - 450) / 24;
    if (k < 0) k = 0;
    double gor = qpsk_gl_from_bits((uint64_t)(0x63f00000u - (uint32_t)((k * 24) << 20)) << 32);
    for (int i = 0; i < 6; i++) {
        r[i] = xi * toverp[k + i] * gor;
        gor *= 0x1p-24;
    }
    for (int i = 0; i < 3; i++) {
        s = (r[i] + big) - big;
        sum += s;
        r[i] -= s;
    }
    t = 0;
    for (int i = 0; i < 6; i++) t += r[5 - i];
    bb = (((((r[0] - t) + r[1]) + r[2]) + r[3]) + r[4]) + r[5];
    s = (t + big) - big;
    sum += s;
    t -= s;
    b = t + bb;
    bb = (t - b) + bb;
    s = (sum + big1) - big1;
    sum -= s;
    *bo = b;
    *bbo = bb;
    *sumo = sum;
}

/* x = n pi/2 + (a + aa) for a finite |x| >= 105414350 (branred.c __branred) */
QPSK_GHD static inline int qpsk_gl_branred(double x, double *a, double *aa)
{
    const double split = 134217729.0, mp2 = -0x1.dde974p-27;
    double b1, bb1, sum1, b2, bb2, sum2;
    x *= 0x1p-600;
    double t = x * split;
    const double x1 = t - (t - x);
    const double x2 = x - x1;
    qpsk_gl_branred_part(x1, &b1, &bb1, &sum1);
    qpsk_gl_branred_part(x2, &b2, &bb2, &sum2);
    double sum = sum1 + sum2;
    double b = b1 + b2;
    double bb = (fabs(b1) > fabs(b2)) ? (b1 - b) + b2 : (b2 - b) + b1;
    if (b > 0.5) {
        b -= 1.0;
        sum += 1.0;
    } else if (b < -0.5) {
        b += 1.0;
        sum -= 1.0;
    }
    double s = b + (bb + bb1 + bb2);
    t = ((b - s) + bb) + (bb1 + bb2);
    b = s * split;
    const double t1 = b - (b - s);
    const double t2 = s - t1;
    b = s * QPSK_GL_HP0;
    bb = (((t1 * QPSK_GL_MP1 - b) + t1 * mp2) + t2 * QPSK_GL_MP1) + (t2 * mp2 + s * QPSK_GL_HP1 + t * QPSK_GL_HP0);
    s = b + bb;
    t = (b - s) + bb;
    *a = s;
    *aa = t;
    return ((int)sum) & 3;
}

QPSK_GHD static inline double qpsk_gl_do_sincos(double a, double da, int n, const double *tab)
{
    const double r = (n & 1) ? qpsk_gl_do_cos(a, da, tab) : qpsk_gl_do_sin(a, da, tab);
    return (n & 2) ? -r : r;
}

QPSK_GHD static inline double qpsk_glibc_sin(double x, const double *tab)
{
    const uint32_t k = (uint32_t)(qpsk_gl_bits(x) >> 32) & 0x7fffffffu;
    double a, da;
    if (k < 0x3e500000u) return x;
    if (k < 0x3feb6000u) return qpsk_gl_do_sin(x, 0.0, tab);
    if (k < 0x400368fdu) return copysign(qpsk_gl_do_cos(QPSK_GL_HP0 - fabs(x), QPSK_GL_HP1, tab), x);
    if (k < 0x419921fbu) {
        const int n = qpsk_gl_reduce_sincos(x, &a, &da);
        return qpsk_gl_do_sincos(a, da, n, tab);
    }
    if (k < 0x7ff00000u) {
        const int n = qpsk_gl_branred(x, &a, &da);
        return qpsk_gl_do_sincos(a, da, n, tab);
    }
    return x / x;
}

QPSK_GHD static inline double qpsk_glibc_cos(double x, const double *tab)
{
    const uint32_t k = (uint32_t)(qpsk_gl_bits(x) >> 32) & 0x7fffffffu;
    double a, da;
    if (k < 0x3e400000u) return 1.0;
    if (k < 0x3feb6000u) return qpsk_gl_do_cos(x, 0.0, tab);
    if (k < 0x400368fdu) {
        const double y = QPSK_GL_HP0 - fabs(x);
        a = y + QPSK_GL_HP1;
        da = (y - a) + QPSK_GL_HP1;
        return qpsk_gl_do_sin(a, da, tab);
    }
    if (k < 0x419921fbu) {
        const int n = qpsk_gl_reduce_sincos(x, &a, &da);
        return qpsk_gl_do_sincos(a, da, n + 1, tab);
    }
    if (k < 0x7ff00000u) {
        const int n = qpsk_gl_branred(x, &a, &da);
        return qpsk_gl_do_sincos(a, da, n + 1, tab);
    }
    return x / x;
}


/* sin and cos of one argument (the Costas NCO needs both), as two calls */
QPSK_GHD static inline void qpsk_glibc_sincos(double x, const double *tab, double *s, double *c)
{
    *s = qpsk_glibc_sin(x, tab);
    *c = qpsk_glibc_cos(x, tab);
}

/* ---- branch-free form for wavefront code ---------------------------------
 * glibc's sin(x) and cos(x) each pick an argument region and then evaluate
 * one do_sin or do_cos; per region the pair needs exactly one do_sin and one
 * do_cos:
 *   |x| < 0.855469   sin = do_sin(x, 0)             cos = do_cos(x, 0)
 *   |x| < 2.426265   sin = +-do_cos(y, hp1)         cos = do_sin(y + hp1, da)
 *                    (y = hp0 - |x|)
 *   otherwise        n, a, da = reduce_sincos / __branred: sin and cos are
 *                    do_sin(a, da) and do_cos(a, da), swapped when n is odd,
 *                    negated by bit 1 of n (sin) and of n + 1 (cos)
 * so every lane evaluates one do_sin and one do_cos on selected arguments and
 * the results are assigned by selects: one instruction stream for the whole
 * wave instead of a branch per region and function.  Only __branred (|x| >=
 * 105414350, a QPSK false lock) stays a branch.  Bit-identical to
 * qpsk_glibc_sin / qpsk_glibc_cos (tools/check_glibc_sin.c -DWITH_PRODUCT). */
QPSK_GHD static inline int qpsk_gl_tab_index_clamped(double u)
{
    /* valid arguments give i <= 109 (4 * 109 = 436); NaN / Inf any bits */
    const uint32_t i = (uint32_t)qpsk_gl_bits(u) << 2;
    return (int)(i < 436u ? i : 436u);
}

QPSK_GHD static inline double qpsk_gl_do_sin_bf(double x, double dx, const double *tab)
{
    const double ty = qpsk_gl_taylor_sin(x, dx);
    const double dxs = x <= 0 ? -dx : dx;
    const double ax = fabs(x);
    const double u = QPSK_GL_BIG + ax;
    const double xr = ax - (u - QPSK_GL_BIG);
    const double xx = xr * xr;
    const double s = xr + fma(xr * xx, fma(xx, QPSK_GL_SN5, QPSK_GL_SN3), dxs);
    const double c = fma(xr, dxs, xx * fma(xx, fma(xx, QPSK_GL_CS6, QPSK_GL_CS4), QPSK_GL_CS2));
    const double *t = tab + qpsk_gl_tab_index_clamped(u);
    const double sn = t[0], ssn = t[1], cs = t[2], ccs = t[3];
    double cor = fma(s, ccs, ssn);
    cor = fma(-c, sn, cor);
    cor = fma(s, cs, cor);
    const double r = copysign(sn + cor, x);
    return ax < 0.126 ? ty : r;
}

QPSK_GHD static inline double qpsk_gl_do_cos_bf(double x, double dx, const double *tab)
{
    const double dxc = x < 0 ? -dx : dx;
    const double ax = fabs(x);
    const double u = QPSK_GL_BIG + ax;
    const double xr = (ax - (u - QPSK_GL_BIG)) + dxc;
    const double xx = xr * xr;
    const double s = fma(xr * xx, fma(xx, QPSK_GL_SN5, QPSK_GL_SN3), xr);
    const double c = xx * fma(xx, fma(xx, QPSK_GL_CS6, QPSK_GL_CS4), QPSK_GL_CS2);
    const double *t = tab + qpsk_gl_tab_index_clamped(u);
    const double sn = t[0], ssn = t[1], cs = t[2], ccs = t[3];
    double cor = fma(-s, ssn, ccs);
    cor = fma(-c, cs, cor);
    cor = fma(-s, sn, cor);
    return cs + cor;
}

/* full = 0: the caller guarantees |x| < 0x1.921fbp+26 (= 105414348, hi word
 * 0x419921fb) or a non-finite x, so __branred is left out (the GPU Costas loop
 * tracks max |theta| and redoes a round with full = 1 if it was exceeded) */
QPSK_GHD static inline void qpsk_glibc_sincos_bf_k(double x, const double *tab, double *s_out, double *c_out,
                                                   int full)
{
    const uint32_t k = (uint32_t)(qpsk_gl_bits(x) >> 32) & 0x7fffffffu;
    double aC, daC;
    int n = qpsk_gl_reduce_sincos(x, &aC, &daC);
    if (full && k >= 0x419921fbu && k < 0x7ff00000u) n = qpsk_gl_branred(x, &aC, &daC);
    const double y = QPSK_GL_HP0 - fabs(x);
    const double aB = y + QPSK_GL_HP1;
    const double daB = (y - aB) + QPSK_GL_HP1;
    const int rA = k < 0x3feb6000u;
    const int rB = k < 0x400368fdu;
    const double xs = rA ? x : (rB ? aB : aC);
    const double dxs = rA ? 0.0 : (rB ? daB : daC);
    const double xc = rA ? x : (rB ? y : aC);
    const double dxc = rA ? 0.0 : (rB ? QPSK_GL_HP1 : daC);
    const double DS = qpsk_gl_do_sin_bf(xs, dxs, tab);
    const double DC = qpsk_gl_do_cos_bf(xc, dxc, tab);
    const int odd = (n & 1) != 0;
    double sC = odd ? DC : DS, cC = odd ? DS : DC;
    sC = (n & 2) ? -sC : sC;
    cC = ((n + 1) & 2) ? -cC : cC;
    double s = rA ? DS : (rB ? copysign(DC, x) : sC);
    double c = rA ? DC : (rB ? DS : cC);
    if (k < 0x3e500000u) s = x;
    if (k < 0x3e400000u) c = 1.0;
    if (k >= 0x7ff00000u) s = c = x - x;   /* glibc: x / x, NaN */
    *s_out = s;
    *c_out = c;
}

#define QPSK_GLIBC_SMALL_LIMIT 0x1.921fbp+26   /* |x| below: qpsk_glibc_sincos_bf_k(full = 0) is exact */

/* ---- split form: two lanes per argument ------------------------------------
 * The do_sin and the do_cos of the branch-free form run on two lanes of the
 * same wave (the GPU Costas loop: lane l and lane l + 32 carry the same
 * stream), each with its own layout of the table so that one code path
 * serves both:
 *   h = 0 (do_sin):  {ccs, ssn, sn, cs}     cor = ((s*T0 + T1) - c*T2) + s*T3
 *   h = 1 (do_cos):  {-ssn, ccs, cs, -sn}   r = T2 + cor
 * (s*(-ssn) + ccs rounds as ccs - s*ssn, an fma with a negated operand is
 * the same rounding), and the sin-only terms fold in as +0 / x*0 where the
 * cos has none (exact: those terms add +0 to a value that is never -0).
 * Every step equals qpsk_gl_do_sin_bf (h = 0) / qpsk_gl_do_cos_bf (h = 1);
 * tools/check_glibc_sin.c -DWITH_PRODUCT checks the assembled pair. */
QPSK_GHD static inline void qpsk_gl_half_tables(const double *tab, int i, double *ts4, double *tc4)
{
    /* entry i of the two layouts from __sincostab entry i = {sn, ssn, cs, ccs} */
    const double sn = tab[4 * i], ssn = tab[4 * i + 1], cs = tab[4 * i + 2], ccs = tab[4 * i + 3];
    ts4[0] = ccs; ts4[1] = ssn; ts4[2] = sn; ts4[3] = cs;
    tc4[0] = -ssn; tc4[1] = ccs; tc4[2] = cs; tc4[3] = -sn;
}

QPSK_GHD static inline double qpsk_gl_do_half(double x, double dx, int h, const double *tabh)
{
    const double ty = qpsk_gl_taylor_sin(x, dx);
    const int flip = h ? (x < 0) : (x <= 0);
    const double d = flip ? -dx : dx;
    const double ax = fabs(x);
    const double u = QPSK_GL_BIG + ax;
    const double xr = (ax - (u - QPSK_GL_BIG)) + (h ? d : 0.0);
    const double xx = xr * xr;
    const double q = xr * xx;
    const double p = fma(xx, QPSK_GL_SN5, QPSK_GL_SN3);
    const double s = (h ? 0.0 : xr) + fma(q, p, h ? xr : d);
    const double c = fma(xr, h ? 0.0 : d, xx * fma(xx, fma(xx, QPSK_GL_CS6, QPSK_GL_CS4), QPSK_GL_CS2));
    const double *t = tabh + qpsk_gl_tab_index_clamped(u);
    double cor = fma(s, t[0], t[1]);
    cor = fma(-c, t[2], cor);
    cor = fma(s, t[3], cor);
    const double r = t[2] + cor;
    return h ? r : (ax < 0.126 ? ty : copysign(r, x));
}

/* the argument of half h (0: do_sin, 1: do_cos) and the region bookkeeping */
typedef struct {
    double xa, dxa;
    int n, rA, rB;
} qpsk_gl_split_arg;

QPSK_GHD static inline qpsk_gl_split_arg qpsk_gl_split_prepare(double x, int h, int full)
{
    qpsk_gl_split_arg g;
    const uint32_t k = (uint32_t)(qpsk_gl_bits(x) >> 32) & 0x7fffffffu;
    double aC, daC;
    g.n = qpsk_gl_reduce_sincos(x, &aC, &daC);
    if (full && k >= 0x419921fbu && k < 0x7ff00000u) g.n = qpsk_gl_branred(x, &aC, &daC);
    const double y = QPSK_GL_HP0 - fabs(x);
    const double aB = y + QPSK_GL_HP1;
    const double daB = (y - aB) + QPSK_GL_HP1;
    g.rA = k < 0x3feb6000u;
    g.rB = k < 0x400368fdu;
    g.xa = g.rA ? x : (g.rB ? (h ? y : aB) : aC);
    g.dxa = g.rA ? 0.0 : (g.rB ? (h ? QPSK_GL_HP1 : daB) : daC);
    return g;
}

/* sin and cos from DS = do_sin and DC = do_cos of the prepared arguments */
QPSK_GHD static inline void qpsk_gl_split_finish(double x, const qpsk_gl_split_arg *g, double DS, double DC,
                                                 double *s_out, double *c_out)
{
    const uint32_t k = (uint32_t)(qpsk_gl_bits(x) >> 32) & 0x7fffffffu;
    /* region A: (DS, DC); B: (+-DC, DS); C: by the parity of n, signs by bits
     * of n and n + 1.  swap and both signs as integer logic, then two selects */
    const int swap = g->rA ? 0 : (g->rB ? 1 : (g->n & 1));
    double s = swap ? DC : DS, c = swap ? DS : DC;
    const uint64_t sgn = 0x8000000000000000ull;
    const uint64_t ns = g->rA ? 0 : (g->rB ? (qpsk_gl_bits(x) & sgn) : ((g->n & 2) ? sgn : 0));
    const uint64_t nc = (g->rA || g->rB) ? 0 : (((g->n + 1) & 2) ? sgn : 0);
    s = qpsk_gl_from_bits(qpsk_gl_bits(s) ^ ns);
    c = qpsk_gl_from_bits(qpsk_gl_bits(c) ^ nc);
    if (k < 0x3e500000u) s = x;
    *s_out = s;
    *c_out = c;
}

/* ---- fast split form (round 4): both halves work on |x| ---------------------
 * For |x| < QPSK_GLIBC_SMALL_LIMIT (or NaN) glibc's pair is odd/even in x bit
 * for bit: sin(x) = sign(x) * sin(|x|), cos(x) = cos(|x|) -- every operation of
 * do_sin, do_cos, TAYLOR_SIN and reduce_sincos maps -x (with -dx) to the exact
 * negative (round-to-nearest is sign-symmetric, and TOINT + k rounds ties to
 * the even k whatever its sign), so the region logic, the dx flips and the
 * sign bookkeeping of the general form run once, on |x|:
 *   |x| < 0.855469:  sin = do_sin(|x|, 0)      cos = do_cos(|x|, 0)
 *   |x| < 2.426265:  sin = do_cos(y, hp1)      cos = do_sin(y + hp1, da)   (y = hp0 - |x|)
 *   otherwise:       n, b, db = reduce_sincos(|x|); sin = do_sin(b, db) / do_cos(b, db)
 *                    by n & 1, signs by bit 1 of n (sin) and of n + 1 (cos)
 * and the sign of x goes onto the sine at the end.  glibc's |x| < 2^-26 (sin =
 * x) and |x| < 2^-27 (cos = 1) shortcuts need no branch: TAYLOR_SIN and the
 * table path round to exactly those values there.
 * The two halves differ only by per-lane constants (qpsk_gl_fs_lane), so they
 * run ONE instruction sequence: with L0 = 1, L1 = 0 (do_sin half) or L0 = 0,
 * L1 = 1 (do_cos half)
 *   xr = fma(d, L1, z)                    do_cos adds dx, do_sin does not
 *   s  = fma(q, p, fma(xr, L1, d*L0)) + xr*L0
 *                                         do_sin: xr + fma(q, p, d); do_cos: fma(q, p, xr)
 *   c  = fma(xr, d*L0, X)                 do_sin: xr*d + X;  do_cos: X
 * (a zero product adds a signed zero to a value that is never -0, so each is
 * the op it replaces bit for bit), and B = y + hp1 * L0 is the do_sin half's
 * y + hp1 and the do_cos half's y.  Each half's result carries the sign its
 * value has in the pair (bit 1 of n + 1 on the do_sin half, of n on the do_cos
 * half, region C only), so after the exchange only the swap (region B, or n
 * odd) and the sign of x remain.  tools/check_glibc_sin.c -DWITH_PRODUCT checks
 * the assembled pair against the real libm. */
typedef struct {
    double L0, L1, hp1L;    /* 1, 0, hp1 on the do_sin half; 0, 1, 0 on the do_cos half */
    uint32_t sgnm;          /* 0x80000000 on the do_sin half (copysign), 0 on the other */
    uint32_t tsh;           /* 1 << 30 on the do_sin half: its sign is bit 1 of n + 1 */
    uint32_t sign;          /* 0x80000000 on both */
    int sin_half;
    /* the fma addends of the polynomials and the reduction (uniform): device
     * code pins them in VGPRs, so no iteration rebuilds them from SGPR halves
     * (a VOP3 op reads one scalar operand) */
    double toint, s4, sn3, cs4;
} qpsk_gl_fs_lane;

QPSK_GHD static inline qpsk_gl_fs_lane qpsk_gl_fs_lane_init(int sin_half)
{
    qpsk_gl_fs_lane k;
    k.L0 = sin_half ? 1.0 : 0.0;
    k.L1 = sin_half ? 0.0 : 1.0;
    k.hp1L = sin_half ? QPSK_GL_HP1 : 0.0;
    k.sgnm = sin_half ? 0x80000000u : 0u;
    k.tsh = sin_half ? 0x40000000u : 0u;
    k.sign = 0x80000000u;
    k.sin_half = sin_half;
    k.toint = QPSK_GL_TOINT;
    k.s4 = QPSK_GL_S4;
    k.sn3 = QPSK_GL_SN3;
    k.cs4 = QPSK_GL_CS4;
    return k;
}

/* hi-word bit helpers: (m & a) | (~m & b), and (v << 5) + base */
QPSK_GHD static inline uint32_t qpsk_gl_bfi(uint32_t m, uint32_t a, uint32_t b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
#else
    return (m & a) | (~m & b);
#endif
}

QPSK_GHD static inline double qpsk_gl_with_hi(double v, uint32_t hi)
{
    return qpsk_gl_from_bits((qpsk_gl_bits(v) & 0xffffffffull) | ((uint64_t)hi << 32));
}

QPSK_GHD static inline uint32_t qpsk_gl_hi(double v) { return (uint32_t)(qpsk_gl_bits(v) >> 32); }

/* the scheduler must not move the rest of the pair ahead of the row's loads */
#if defined(__HIP_DEVICE_COMPILE__)
#define QPSK_GL_SCHED_BARRIER() __builtin_amdgcn_sched_barrier(0)
#else
#define QPSK_GL_SCHED_BARRIER() ((void)0)
#endif

/* This half's value of the pair of x, with the sign it takes in the pair
 * (do_sin on the K->sin_half lanes, do_cos on the others), and *swap: the
 * do_cos half's value is sin(|x|) (region B, or region C with n odd).
 *
 * Region A runs as region C with n = 0: with the high word of 1/hp0 zeroed
 * (a denormal), tt = toint exactly, xn = 0, and reduce_sincos returns
 * (|x|, +0), which are region A's argument and dx bit for bit (-0 * c adds a
 * signed zero to |x| or to +0), while tt's low word gives n = 0 (no swap, no
 * quadrant sign).  The argument selects then have two ways instead of three.
 *
 * Order (round 5): the argument xa and the table row's address come first and
 * the row's four loads are issued before anything else, behind a scheduling
 * barrier, so the LDS round trip runs under dx, the quadrant logic and both
 * polynomials instead of after them (tools/gl_costas_probe.hip). */
QPSK_GHD static inline double qpsk_gl_fs_pair(double x, const qpsk_gl_fs_lane *K, const double *tabh, int *swap)
{
    const double ax = fabs(x);
    const int rA = ax < 0x1.b6p-1;                   /* hi word < 0x3feb6000 */
    const int rB = ax < 0x1.368fdp+1;                /* hi word < 0x400368fd */
    const int rBo = rB && !rA;                       /* region B proper */
    /* region C: reduce_sincos(|x|); region A: the same with n = 0 */
    const uint64_t hpb = qpsk_gl_bits(QPSK_GL_HPINV);
    const double hpinv = qpsk_gl_from_bits(rA ? (hpb & 0xffffffffull) : hpb);
    const double tt = fma(ax, hpinv, K->toint);
    const double xn = tt - QPSK_GL_TOINT;
    double y = fma(-xn, QPSK_GL_MP1, ax);
    y = fma(-xn, QPSK_GL_MP2, y);
    const double t2 = fma(-xn, QPSK_GL_PP3, y);
    const double b = fma(-xn, QPSK_GL_PP4, t2);
    /* region B */
    const double yb = QPSK_GL_HP0 - ax;
    const double xb = yb + K->hp1L;
    const double xa = rBo ? xb : b;
    /* the table row: u = BIG + |xa| (valid arguments give node <= 109; NaN
     * any bits, still inside the table) */
    const double axa = fabs(xa);
    const double u = QPSK_GL_BIG + axa;
    const uint32_t node = (uint32_t)qpsk_gl_bits(u) & 127u;
#if defined(__HIP_DEVICE_COMPILE__)
    /* the table is in LDS: a 32-bit LDS address, node * 32 B + base in one op */
    typedef __attribute__((address_space(3))) const double lds_double;
    uint32_t addr;
    asm("v_lshl_add_u32 %0, %1, 5, %2"
        : "=v"(addr)
        : "v"(node), "v"((uint32_t)(uintptr_t)(lds_double *)tabh));
    lds_double *tb = (lds_double *)(uintptr_t)addr;
#else
    const double *tb = tabh + 4 * node;
#endif
    const double T0 = tb[0], T1 = tb[1], T2 = tb[2], T3 = tb[3];
    QPSK_GL_SCHED_BARRIER();
    double db = fma(-xn, QPSK_GL_PP3, y - t2);
    db = db + fma(-xn, QPSK_GL_PP4, t2 - b);
    const double dB = (yb - xb) + QPSK_GL_HP1;
    const double dxa = rBo ? dB : db;
    /* n << 30: bit 31 = bit 1 of n, bit 30 = bit 0 (0 in region A) */
    const uint32_t tn = (uint32_t)qpsk_gl_bits(tt) << 30;
    const uint32_t t = rBo ? 0u : tn;
    *swap = rBo ? 1 : (int)(tn >> 30) & 1;
    /* TAYLOR_SIN (qpsk_gl_taylor_sin) with the pinned addend */
    const double ta = xa * xa;
    double tp = fma(ta, QPSK_GL_S5, K->s4);
    tp = fma(ta, tp, QPSK_GL_S3);
    tp = fma(ta, tp, QPSK_GL_S2);
    tp = fma(ta, tp, QPSK_GL_S1);
    const double ty = xa + fma(ta, fma(tp, xa, -(0.5 * dxa)), dxa);
    /* d = dx, negated when xa < 0 (xa is never -0): the sign of xa XORed in */
    const double d = qpsk_gl_with_hi(dxa, qpsk_gl_hi(dxa) ^ (qpsk_gl_hi(xa) & K->sign));
    const double xr = fma(d, K->L1, axa - (u - QPSK_GL_BIG));
    const double xx = xr * xr;
    const double q = xr * xx;
    const double p = fma(xx, QPSK_GL_SN5, K->sn3);
    const double dl = d * K->L0;
    const double s = fma(q, p, fma(xr, K->L1, dl)) + xr * K->L0;
    const double c = fma(xr, dl, xx * fma(xx, fma(xx, QPSK_GL_CS6, K->cs4), QPSK_GL_CS2));
    double cor = fma(s, T0, T1);
    cor = fma(-c, T2, cor);
    cor = fma(s, T3, cor);
    const double r = T2 + cor;
    /* do_sin: copysign(r, xa) (r > 0); do_sin below 0.126: TAYLOR_SIN */
    double v = qpsk_gl_with_hi(r, qpsk_gl_bfi(K->sgnm, qpsk_gl_hi(xa), qpsk_gl_hi(r)));
    if (K->sin_half && axa < 0.126) v = ty;
    /* the pair's sign of this value (region C) */
    return qpsk_gl_with_hi(v, qpsk_gl_hi(v) ^ ((t + K->tsh) & K->sign));
}

/* sin and cos of x from the do_sin half's value VS and the do_cos half's VC */
QPSK_GHD static inline void qpsk_gl_fs_finish(double x, int swap, double VS, double VC, const qpsk_gl_fs_lane *K,
                                              double *s_out, double *c_out)
{
    const double s = swap ? VC : VS, c = swap ? VS : VC;
    *s_out = qpsk_gl_with_hi(s, qpsk_gl_hi(s) ^ (qpsk_gl_hi(x) & K->sign));
    *c_out = c;
}

/* host form of the fast split pair (both halves in one thread), for the checker */
QPSK_GHD static inline void qpsk_glibc_sincos_fs_host(double x, const double *tabs, const double *tabc,
                                                      double *s_out, double *c_out)
{
    const qpsk_gl_fs_lane k0 = qpsk_gl_fs_lane_init(1), k1 = qpsk_gl_fs_lane_init(0);
    int w0, w1;
    const double VS = qpsk_gl_fs_pair(x, &k0, tabs, &w0);
    const double VC = qpsk_gl_fs_pair(x, &k1, tabc, &w1);
    qpsk_gl_fs_finish(x, w0, VS, VC, &k0, s_out, c_out);
}

/* host form of the split evaluation (both halves in one thread), for the checker */
QPSK_GHD static inline void qpsk_glibc_sincos_split_host(double x, const double *tabs, const double *tabc,
                                                         double *s_out, double *c_out)
{
    const qpsk_gl_split_arg g0 = qpsk_gl_split_prepare(x, 0, 1), g1 = qpsk_gl_split_prepare(x, 1, 1);
    const double DS = qpsk_gl_do_half(g0.xa, g0.dxa, 0, tabs);
    const double DC = qpsk_gl_do_half(g1.xa, g1.dxa, 1, tabc);
    qpsk_gl_split_finish(x, &g0, DS, DC, s_out, c_out);
}

QPSK_GHD static inline void qpsk_glibc_sincos_bf(double x, const double *tab, double *s_out, double *c_out)
{
    qpsk_glibc_sincos_bf_k(x, tab, s_out, c_out, 1);
}

#endif /* QPSK_GLIBC_TRIG_H */
