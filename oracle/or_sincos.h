/*
 * or_sincos.h -- ORACLE copy of the portable double sin+cos used as the
 * deterministic stand-in for .NET Math.Cos/Math.Sin (CostasLoopQpsk.cs:69-70),
 * and of the glibc sinf/cosf restatement that MathF.Cos/MathF.Sin
 * (Band-Edge Filter.cs:108-109) call on Linux (second half of this file).
 *
 * TEST INFRASTRUCTURE ONLY.  The product carries its own copy of the same
 * published algorithm (qpsk-modulator-demodulator_amd/csrc/qpsk_sincos.h); a
 * CPU test sweeps both and requires bitwise-identical results.
 *
 * Algorithm: Cody-Waite reduction by pi/256 with a two-part constant (fma;
 * the integer multiple comes from the 1.5*2^52 shifter, which also yields the
 * table index), a 512-entry table of correctly rounded sin/cos(k pi/256)
 * (tools/gen_sincos_table.py), degree-5/6 Taylor polynomials for the residual
 * |r| <= pi/512 and angle addition with the table value added last.
 * Accuracy <= 1 ulp (table rounding + one final rounding).
 * Every operation is an IEEE-754 double op or an explicit fma(), so the result
 * is bit-identical on any IEEE host and on gfx950 (v_fma_f64 is correctly
 * rounded).  Compile with -ffp-contract=off.
 */
#ifndef OR_SINCOS_H
#define OR_SINCOS_H
#include <math.h>
#include <stdint.h>
#include "or_sincos_table.h"

/* [2k] = sin(k pi/256), [2k+1] = cos(k pi/256), k < 512: correctly rounded
 * double + float tail (tools/gen_sincos_table.py) */
static const double or_sincos_table[1024] = { OR_SINCOS_TAB_VALUES_HI };
static const double or_sincos_table_lo[1024] = { OR_SINCOS_TAB_VALUES_LO };

/* argument the table reduction accepts: |x| <= 2^40 (or NaN).  Up to there
 * k = rint(x*256/pi) < 2^49 and x - k*P1 is a multiple of 2^-59 below 2^-6
 * (so the first fma is exact); the second part leaves k*(pi/256 - P1 - P2),
 * below 2^-106 for |x| <= 8 (the Costas phase in lock) and 2^-69 at 2^40.
 * Larger |x| and +-Inf are pre-reduced with fmod (Inf -> NaN).  The Costas
 * loop's theta leaves [-pi, pi] only once its freq passes pi (a QPSK false
 * lock at a multiple of pi/2 per symbol): theta then grows by ~freq per
 * symbol, which a sustained run reaches within a few calls. */
static inline double or_sincos_arg(double x)
{
    return fabs(x) > 0x1p40 ? fmod(x, 6.28318530717958647693) : x;
}

/* sin and cos of x, |x| <= 2^40 or NaN, given the 512-entry table (any address
 * space: the GPU kernels pass a copy staged in LDS).  Straight-line: the GPU
 * Costas loop is issue-bound and every instruction costs issue slots.  NaN
 * propagates (any table index gives NaN). */
static inline void or_sincos_tab_core(double x, const double *tab, const double *lo,
                                           double *s, double *c)
{
    const double INV = 0x1.45f306dc9c883p+6;       /* 256/pi */
    const double SH = 0x1.8p+52;                   /* 1.5*2^52: ulp 1 */
    const double P1 = 0x1.921fb54442d18p-7;        /* pi/256 rounded to double */
    const double P2 = 0x1.1a62633145c07p-61;       /* next 53 bits */
    const double S3 = -0x1.5555555555555p-3, S5 = 0x1.1111111111111p-7;    /* -1/6, 1/120 */
    const double C4 = 0x1.5555555555555p-5, C6 = -0x1.6c16c16c16c17p-10;  /* 1/24, -1/720 */
    /* kb = fma(x, 256/pi, 1.5*2^52) rounds the exact product to an integer
     * (ties to even), so k = kb - 1.5*2^52 = rint(x*256/pi) exactly
     * (|x| <= 2^40) and the low mantissa bits of kb are k mod 512 in two's
     * complement: the table index without a separate rint */
    union { double d; unsigned long long u; } kb;
    kb.d = fma(x, INV, SH);
    const double k = kb.d - SH;
    double r = fma(-k, P1, x);                     /* Cody-Waite: |r| <= pi/512 */
    r = fma(-k, P2, r);
    const unsigned i = (unsigned)(kb.u & 511u) * 2u;
    const double ts = tab[i], tc = tab[i + 1];
    const double ls = lo[i], lc = lo[i + 1];
    /* sin r = r + r^3(-1/6 + r^2/120), cos r - 1 = r^2(-1/2 + r^2/24 - r^4/720):
     * truncation < 1e-19 relative for |r| <= pi/512 */
    const double z = r * r;
    const double r3p = (r * z) * fma(z, S5, S3);          /* sin r - r */
    const double cm = z * fma(z, fma(z, C6, C4), -0.5);   /* cos r - 1 */
    /* angle addition, small terms first: sin x = ts + [tc r + (tc r3p + ts cm + ls)],
     * one significant rounding in the bracket and one in the final add: <= 1 ulp */
    *s = ts + fma(tc, r, fma(tc, r3p, fma(ts, cm, ls)));
    *c = tc + fma(-ts, r, fma(-ts, r3p, fma(tc, cm, lc)));
}

/* any x: the pre-reduction branch, then the table reduction */
static inline void or_sincos_tab(double x, const double *tab, const double *lo, double *s,
                                      double *c)
{
    if (__builtin_expect(fabs(x) > 0x1p40, 0)) x = or_sincos_arg(x);
    or_sincos_tab_core(x, tab, lo, s, c);
}

static inline void or_sincos(double x, double *s, double *c)
{
    or_sincos_tab(x, or_sincos_table, or_sincos_table_lo, s, c);
}

/* ---------------------------------------------------------------------------
 * MathF.Sin / MathF.Cos (Band-Edge Filter.cs:108-109): .NET calls the C
 * runtime's sinf/cosf, i.e. glibc on a Linux host.  Restated here in glibc's
 * own structure (glibc 2.35 sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c,
 * sincosf.h, sincosf_data.c; the ARM optimized-routines algorithm), as its
 * x86-64 FMA ifunc variant evaluates it (every a*b+c contracted into one fma).
 * tools/check_glibc_sincosf.c compares or_sinf/or_cosf with the real glibc on
 * all 2^32 inputs (bit-identical, NaNs as NaN); the product's fused form is
 * csrc/qpsk_sincosf.h, checked against these by tests/test_oracle.py.
 * ------------------------------------------------------------------------- */
typedef struct {
    double sign[4];
    double hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
} or_sincosf_t;

static const or_sincosf_t or_sincosf_table[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0,
     -0x1.ffffffd0c621cp-2, 0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10,
     0x1.99343027bf8c3p-16, -0x1.555545995a603p-3, 0x1.1107605230bc4p-7,
     -0x1.994eb3774cf24p-13},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0,
     0x1.ffffffd0c621cp-2, -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10,
     -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3, 0x1.1107605230bc4p-7,
     -0x1.994eb3774cf24p-13}};

/* 4/pi in 32-bit windows, 8 new bits per entry (sincosf_data.c __inv_pio4) */
static const uint32_t or_inv_pio4[24] = {
    0xa2, 0xa2f9, 0xa2f983, 0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
    0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
    0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};

static inline uint32_t or_asuint(float f)
{
    union { float f; uint32_t u; } v;
    v.f = f;
    return v.u;
}
static inline uint32_t or_abstop12(float x) { return (or_asuint(x) >> 20) & 0x7ff; }

static inline float or_sinf_poly(double x, double x2, const or_sincosf_t *p, int n)
{
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = fma(x2, p->s3, p->s2);
        double x7 = x3 * x2;
        double s = fma(x3, p->s1, x);
        return (float)fma(x7, s1, s);
    }
    double x4 = x2 * x2;
    double c2 = fma(x2, p->c4, p->c3);
    double c1 = fma(x2, p->c1, p->c0);
    double x6 = x4 * x2;
    double c = fma(x4, p->c2, c1);
    return (float)fma(x6, c2, c);
}

static inline double or_reduce_fast(double x, const or_sincosf_t *p, int *np)
{
    double r = x * p->hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return fma(-(double)n, p->hpi, x);
}

static inline double or_reduce_large(uint32_t xi, int *np)
{
    const uint32_t *arr = &or_inv_pio4[(xi >> 26) & 15];
    int shift = (xi >> 23) & 7;
    uint64_t n, res0, res1, res2;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    res0 = (uint32_t)(xi * arr[0]);
    res1 = (uint64_t)xi * arr[4];
    res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    *np = (int)n;
    return (double)(int64_t)res0 * 0x1.921FB54442D18p-62;
}

static inline float or_sinf(float y)
{
    double x = y, s;
    int n;
    const or_sincosf_t *p = &or_sincosf_table[0];
    if (or_abstop12(y) < or_abstop12(0x1.921FB6p-1f)) {
        s = x * x;
        if (or_abstop12(y) < or_abstop12(0x1p-12f)) return y;
        return or_sinf_poly(x, s, p, 0);
    } else if (or_abstop12(y) < or_abstop12(120.0f)) {
        x = or_reduce_fast(x, p, &n);
        s = p->sign[n & 3];
        if (n & 2) p = &or_sincosf_table[1];
        return or_sinf_poly(x * s, x * x, p, n);
    } else if (or_abstop12(y) < or_abstop12(INFINITY)) {
        uint32_t xi = or_asuint(y);
        int sign = xi >> 31;
        x = or_reduce_large(xi, &n);
        s = p->sign[(n + sign) & 3];
        if ((n + sign) & 2) p = &or_sincosf_table[1];
        return or_sinf_poly(x * s, x * x, p, n);
    }
    return (y - y) / (y - y);
}

static inline float or_cosf(float y)
{
    double x = y, s;
    int n;
    const or_sincosf_t *p = &or_sincosf_table[0];
    if (or_abstop12(y) < or_abstop12(0x1.921FB6p-1f)) {
        double x2 = x * x;
        if (or_abstop12(y) < or_abstop12(0x1p-12f)) return 1.0f;
        return or_sinf_poly(x, x2, p, 1);
    } else if (or_abstop12(y) < or_abstop12(120.0f)) {
        x = or_reduce_fast(x, p, &n);
        s = p->sign[n & 3];
        if (n & 2) p = &or_sincosf_table[1];
        return or_sinf_poly(x * s, x * x, p, n ^ 1);
    } else if (or_abstop12(y) < or_abstop12(INFINITY)) {
        uint32_t xi = or_asuint(y);
        int sign = xi >> 31;
        x = or_reduce_large(xi, &n);
        s = p->sign[(n + sign) & 3];
        if ((n + sign) & 2) p = &or_sincosf_table[1];
        return or_sinf_poly(x * s, x * x, p, n ^ 1);
    }
    return (y - y) / (y - y);
}

/* the FLL's float trig in the oracle's portable mode */
static inline void or_sincosf(float x, float *s, float *c)
{
    *c = or_cosf(x);
    *s = or_sinf(x);
}
#endif
