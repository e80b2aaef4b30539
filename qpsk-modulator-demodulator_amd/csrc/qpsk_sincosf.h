/*
 * qpsk_sincosf.h -- PRODUCT float sin+cos for the Band-Edge FLL's NCO
 * (MathF.Cos / MathF.Sin of the float phase, Band-Edge Filter.cs:108-109).
 *
 * .NET's MathF.Sin/Cos call the C runtime's sinf/cosf; on a Linux x86-64 host
 * that is glibc.  This header restates glibc's published single-precision
 * algorithm (glibc 2.35 sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h,
 * sincosf_data.c -- the ARM optimized-routines sinf/cosf, unchanged since glibc
 * 2.28) in the form glibc's x86-64 FMA ifunc variant (s_sinf-fma.c, selected on
 * every AVX2+FMA host, the EPYC GPU hosts included) evaluates it: every a*b+c
 * of the polynomial and of the pi/2 reduction contracted into one fma.
 *
 *   |y| < pi/4 (by the top 12 bits): no reduction; |y| < 2^-12: sin = y, cos = 1
 *   |y| < 120: n = round(y * 2/pi) from a 2^24-scaled product, x = y - n*pi/2 (fma)
 *   finite:    Payne-Hanek with 4/pi to 192 bits (reduce_large)
 *   Inf/NaN:   NaN
 * then sin/cos polynomials in double on x (signs and the cos table by quadrant)
 * and one rounding to float.
 *
 * tools/check_glibc_sincosf.c compares this restatement (through the oracle's
 * copy, oracle/or_sincos.h) with the real glibc sinf and cosf on ALL 2^32 float
 * inputs: bit-identical (NaNs as NaN).  tests/test_oracle.py runs it and
 * requires the product and oracle copies to agree.
 *
 * Host + device; compile with -ffp-contract=off (the fma calls are explicit).
 *
 * Licence: the algorithm and polynomial constants are those of glibc's
 * sinf/cosf (contributed by Arm Ltd from its optimized-routines library,
 * Copyright (c) 2018 Arm Ltd; LGPL-2.1-or-later in glibc, MIT OR Apache-2.0
 * WITH LLVM-exception in optimized-routines).  Pinned to glibc 2.35
 * (tests/test_oracle.py GLIBC_PIN).
 */
#ifndef QPSK_SINCOSF_H
#define QPSK_SINCOSF_H
#include <math.h>
#include <stdint.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define QPSK_HDF __host__ __device__
#else
#define QPSK_HDF
#endif

/* floor(2^(8k+8) * 2/pi) mod 2^32: 32-bit windows of 2/pi, 8 new bits each */
#define QPSK_INV_PIO4_BITS                                                               \
    0xa2u, 0xa2f9u, 0xa2f983u, 0xa2f9836eu, 0xf9836e4eu, 0x836e4e44u, 0x6e4e4415u,       \
        0x4e441529u, 0x441529fcu, 0x1529fc27u, 0x29fc2757u, 0xfc2757d1u, 0x2757d1f5u,    \
        0x57d1f534u, 0xd1f534ddu, 0xf534ddc0u, 0x34ddc0dbu, 0xddc0db62u, 0xc0db6295u,    \
        0xdb629599u, 0x6295993cu, 0x95993c43u, 0x993c4390u, 0x3c439041u

QPSK_HDF static inline uint32_t qpsk_f32_bits(float f)
{
    union { float f; uint32_t u; } v;
    v.f = f;
    return v.u;
}

/* Payne-Hanek reduction of a finite |y| >= 120 (bits u): returns x in
 * [-pi/4, pi/4] and n with y = x + n*pi/2 (mod 2pi, before the sign) */
QPSK_HDF static inline double qpsk_sincosf_reduce_large(uint32_t u, int *np)
{
    const uint32_t inv[24] = {QPSK_INV_PIO4_BITS};
    const uint32_t *arr = inv + ((u >> 26) & 15);
    const int shift = (u >> 23) & 7;
    uint32_t m = ((u & 0xffffffu) | 0x800000u) << shift;
    uint64_t r0 = (uint64_t)(uint32_t)(m * arr[0]);          /* low 32 bits only */
    const uint64_t r1 = (uint64_t)m * arr[4];
    const uint64_t r2 = (uint64_t)m * arr[8];
    r0 = (r2 >> 32) | (r0 << 32);
    r0 += r1;
    const uint64_t n = (r0 + (1ull << 61)) >> 62;
    r0 -= n << 62;
    *np = (int)n;
    return (double)(int64_t)r0 * 0x1.921FB54442D18p-62;      /* pi * 2^-62 */
}

/* sin(y), cos(y) as glibc 2.35's sinf(y), cosf(y) return them.  FULL = 0 skips
 * the |y| >= 120 branch (the caller guarantees |y| < 120 or NaN). */
#define QPSK_SINCOSF_BODY(FULL)                                                          \
    const uint32_t u = qpsk_f32_bits(y);                                                 \
    const uint32_t top = (u >> 20) & 0x7ffu;                                             \
    double x = (double)y;                                                                \
    int n = 0, q = 0;                                                                    \
    if (top < 0x3f4u) {                      /* abstop12(pi/4) */                        \
        if (top < 0x398u) {                  /* abstop12(2^-12) */                       \
            *s = y;                                                                      \
            *c = 1.0f;                                                                   \
            return;                                                                      \
        }                                                                                \
    } else if (top < 0x42fu) {               /* abstop12(120) */                         \
        const double r = x * 0x1.45F306DC9C883p+23;                /* 2/pi * 2^24 */     \
        n = ((int32_t)r + 0x800000) >> 24;                                               \
        x = fma(-(double)n, 0x1.921FB54442D18p0, x);               /* y - n*pi/2 */      \
        q = n;                                                                           \
    } else if (FULL && top < 0x7f8u) {       /* finite: Payne-Hanek */                   \
        x = qpsk_sincosf_reduce_large(u, &n);                                            \
        q = n + (int)(u >> 31);                                                          \
    } else {                                                                             \
        const float nan_ = (y - y) / (y - y);                                            \
        *s = nan_;                                                                       \
        *c = nan_;                                                                       \
        return;                                                                          \
    }                                                                                    \
    const double x2 = x * x;                                                             \
    const double xs = ((q + 1) & 2) ? -x : x;   /* sign[q & 3] = {1, -1, -1, 1} */       \
    /* sin polynomial (sinf_poly, n even) */                                             \
    const double x3 = xs * x2;                                                           \
    const double s1 = fma(x2, -0x1.994eb3774cf24p-13, 0x1.1107605230bc4p-7);             \
    const double x7 = x3 * x2;                                                           \
    const double sp = fma(x7, s1, fma(x3, -0x1.555545995a603p-3, xs));                   \
    /* cos polynomial (sinf_poly, n odd); the second table negates it */                 \
    const double x4 = x2 * x2;                                                           \
    const double c2 = fma(x2, 0x1.99343027bf8c3p-16, -0x1.6c087e89a359dp-10);            \
    const double c1 = fma(x2, -0x1.ffffffd0c621cp-2, 0x1p0);                             \
    const double x6 = x4 * x2;                                                           \
    double cp = fma(x6, c2, fma(x4, 0x1.55553e1068f19p-5, c1));                          \
    if (q & 2) cp = -cp;                                                                 \
    const float fs = (float)sp, fc = (float)cp;                                          \
    *s = (n & 1) ? fc : fs;                                                              \
    *c = (n & 1) ? fs : fc;

QPSK_HDF static inline void qpsk_sincosf_glibc(float y, float *s, float *c)
{
    QPSK_SINCOSF_BODY(1)
}

/* |y| < 120 or NaN (the FLL phase after its 2pi wrap) */
QPSK_HDF static inline void qpsk_sincosf_glibc_small(float y, float *s, float *c)
{
    QPSK_SINCOSF_BODY(0)
}
#undef QPSK_SINCOSF_BODY

/* Branch-free form for |y| < 120 or NaN (the FLL phase after its 2pi wrap),
 * for wavefront code: the pi/2 reduction always runs.  Below pi/4 it yields
 * n = 0 and x = y exactly (y*2/pi*2^24 < 2^23, and fma(-0, pi/2, y) == y), and
 * below 2^-12 the polynomials round to y and 1 exactly (y = -0 aside, which is
 * kept by a select), so it returns what the branches return (tools/check_glibc_sincosf.c checks every such input). */
/* The branch-free body.  SIGNV is 0x80000000; a device caller may pass it in a
 * register it pinned once (asm "+v"), so the sign logic compiles to 3-input
 * v_bitop3_b32 ops that cannot take a literal. */
QPSK_HDF static inline void qpsk_sincosf_glibc_fast_k(float y, float *s, float *c, uint32_t SIGNV)
{
    const double r = (double)y * 0x1.45F306DC9C883p+23;
    const int n = ((int32_t)r + 0x800000) >> 24;
    const double x = fma(-(double)n, 0x1.921FB54442D18p0, (double)y);
    const double x2 = x * x;
    /* The quadrant logic as bit operations on n (fewer instructions on the
     * FLL's per-sample chain than compares and selects; the same bits).
     * t1 = n << 30 holds bit 1 of n in the sign position, t1 + 2^30 bit 1 of
     * n + 1.  xs = -x when (n + 1) & 2: that bit XORed into x's sign */
    const uint32_t t1 = (uint32_t)n << 30;
    union { double d; uint64_t u; } xb;
    xb.d = x;
    const uint32_t xhi = (uint32_t)(xb.u >> 32) ^ ((t1 + 0x40000000u) & SIGNV);
    xb.u = ((uint64_t)xhi << 32) | (uint32_t)xb.u;
    const double xs = xb.d;
    const double x3 = xs * x2;
    const double s1 = fma(x2, -0x1.994eb3774cf24p-13, 0x1.1107605230bc4p-7);
    const double x7 = x3 * x2;
    const double sp = fma(x7, s1, fma(x3, -0x1.555545995a603p-3, xs));
    const double x4 = x2 * x2;
    const double c2 = fma(x2, 0x1.99343027bf8c3p-16, -0x1.6c087e89a359dp-10);
    const double c1 = fma(x2, -0x1.ffffffd0c621cp-2, 0x1p0);
    const double x6 = x4 * x2;
    const double cp = fma(x6, c2, fma(x4, 0x1.55553e1068f19p-5, c1));
    /* glibc negates cp when n & 2; rounding to float is sign-symmetric, so the
     * sign goes onto the float (bit 1 of n, i.e. t1's sign bit).  sin(-0) must
     * stay -0 (glibc returns y below 2^-12); the polynomial's fma(-0 * S1, -0)
     * is +0.  Then sin/cos swap when n is odd: a bit-select on the mask
     * -(n & 1) (a sign-extended bit-field extract on the device). */
    const uint32_t fcb = qpsk_f32_bits((float)cp) ^ (t1 & SIGNV);
    const uint32_t fsb = y == 0.0f ? qpsk_f32_bits(y) : qpsk_f32_bits((float)sp);
    union { uint32_t u; float f; } so, co;
#if defined(__HIP_DEVICE_COMPILE__)
    /* one mask, two bit-field inserts (the compiler's own form of the select
     * builds both -(n & 1) and its complement) */
    uint32_t odd;
    asm("v_bfe_i32 %2, %3, 0, 1\n\tv_bfi_b32 %0, %2, %4, %5\n\tv_bfi_b32 %1, %2, %5, %4"
        : "=&v"(so.u), "=&v"(co.u), "=&v"(odd)
        : "v"(n), "v"(fcb), "v"(fsb));
#else
    const uint32_t odd = 0u - ((uint32_t)n & 1u);
    so.u = (fcb & odd) | (fsb & ~odd);
    co.u = (fsb & odd) | (fcb & ~odd);
#endif
    *s = so.f;
    *c = co.f;
}

QPSK_HDF static inline void qpsk_sincosf_glibc_fast(float y, float *s, float *c)
{
    qpsk_sincosf_glibc_fast_k(y, s, c, 0x80000000u);
}

/* Lane-split form for |y| < 120 or NaN, y != -0 (the FLL's kept phases, which
 * are never -0 there: qpsk_fll.hip).  Two lanes share one argument: the "sin
 * lane" evaluates glibc's sin polynomial, the "cos lane" its cos polynomial,
 * through ONE instruction sequence with per-lane coefficients, and each then
 * takes the other's result (a DPP swap on the device).
 *
 *   sin lane: m = x,  u = fma(m, 1, -0) = x,            v = m*x2 = x3, w = x7,
 *             fma(v, S0, u), fma(x2, S2, S1)             -> glibc's sp
 *   cos lane: m = x2, u = fma(m, C0, 1) = c1,           v = m*x2 = x4, w = x6,
 *             fma(v, C1, u), fma(x2, C3, C2)             -> glibc's cp
 *
 * The polynomial runs on the unsigned reduced x.  glibc's sign placement (on
 * xs for the sine, on cp for the cosine) is the same bits after the rounding:
 * each op of the odd polynomial maps -x to the exact negative of its result
 * and round-to-nearest is sign-symmetric; x = 0 only for y = +-0, and +0 gives
 * +0 either way.  Quadrant n: the sine value carries the sign of bit 1 of n + 1
 * and goes to sin(y) when n is even, the cosine value the sign of bit 1 of n
 * and goes to sin(y) when n is odd.  With t = (n + T) << 30 (T = 1 on sin
 * lanes, 0 on cos lanes) bit 31 of t is the lane's sign and bit 30 says
 * whether the lane's own value is sin(y) (1) or cos(y) (0).
 * tools/check_glibc_sincosf.c checks both lanes' views on every input. */
struct qpsk_sincosf_lane {
    double q, r, k1, k2, k3;   /* per-lane coefficients */
    uint32_t tsh;              /* T << 30 */
    int sin_lane;
};

QPSK_HDF static inline struct qpsk_sincosf_lane qpsk_sincosf_lane_init(int sin_lane)
{
    struct qpsk_sincosf_lane k;
    k.sin_lane = sin_lane;
    k.q = sin_lane ? 1.0 : -0x1.ffffffd0c621cp-2;
    k.r = sin_lane ? -0.0 : 1.0;
    k.k1 = sin_lane ? -0x1.555545995a603p-3 : 0x1.55553e1068f19p-5;
    k.k2 = sin_lane ? 0x1.1107605230bc4p-7 : -0x1.6c087e89a359dp-10;
    k.k3 = sin_lane ? -0x1.994eb3774cf24p-13 : 0x1.99343027bf8c3p-16;
    k.tsh = sin_lane ? 0x40000000u : 0u;
    return k;
}

/* The lane's own value (sign applied) and t; m is the lane's polynomial
 * argument, chosen by the caller's select (x on sin lanes, x2 on cos lanes) */
#define QPSK_SINCOSF_SPLIT_OWN(y, K, SIGNV, M_SELECT, own, t)                             \
    do {                                                                                  \
        const double yd_ = (double)(y);                                                   \
        /* glibc's ((int32_t)(yd * 2^24 * 2/pi) + 0x800000) >> 24 with the 2^23 folded   \
         * into the product's rounding: the same n for every |y| < 120 (all 2^32 inputs \
         * checked, tools/check_glibc_sincosf.c), one integer add fewer */              \
        const double r_ = fma(yd_, 0x1.45F306DC9C883p+23, 0x1p23);                        \
        const int n_ = (int32_t)r_ >> 24;                                                 \
        const double x_ = fma(-(double)n_, 0x1.921FB54442D18p0, yd_);                    \
        const double x2_ = x_ * x_;                                                       \
        const double m_ = M_SELECT(x_, x2_);                                              \
        const double u_ = fma(m_, (K).q, (K).r);                                          \
        const double v_ = m_ * x2_;                                                       \
        const double w_ = v_ * x2_;                                                       \
        const double a_ = fma(v_, (K).k1, u_);                                            \
        const double b_ = fma(x2_, (K).k3, (K).k2);                                       \
        const double p_ = fma(w_, b_, a_);                                                \
        (t) = ((uint32_t)n_ << 30) + (K).tsh;                                             \
        (own) = qpsk_f32_bits((float)p_) ^ ((t) & (SIGNV));                               \
    } while (0)

#define QPSK_SINCOSF_HOST_SELECT(x, x2) (k.sin_lane ? (x) : (x2))
QPSK_HDF static inline uint32_t qpsk_sincosf_split_own(float y, struct qpsk_sincosf_lane k, uint32_t *t)
{
    uint32_t own, tt;
    QPSK_SINCOSF_SPLIT_OWN(y, k, 0x80000000u, QPSK_SINCOSF_HOST_SELECT, own, tt);
    *t = tt;
    return own;
}
#undef QPSK_SINCOSF_HOST_SELECT

/* own = this lane's value, other = the partner lane's */
QPSK_HDF static inline void qpsk_sincosf_split_pick(uint32_t own, uint32_t other, uint32_t t, float *s, float *c)
{
    const uint32_t m = 0u - ((t >> 30) & 1u);
    union { uint32_t u; float f; } so, co;
    so.u = (own & m) | (other & ~m);
    co.u = (other & m) | (own & ~m);
    *s = so.f;
    *c = co.f;
}
#endif
