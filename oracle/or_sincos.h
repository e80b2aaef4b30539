/*
 * or_sincos.h -- ORACLE copy of the portable double/float sin+cos used as the
 * deterministic stand-in for .NET Math.Cos/Math.Sin (CostasLoopQpsk.cs:69-70)
 * and MathF.Cos/MathF.Sin (Band-Edge Filter.cs:108-109).
 *
 * TEST INFRASTRUCTURE ONLY.  The product carries its own copy of the same
 * published algorithm (qpsk-modulator-demodulator_amd/csrc/qpsk_sincos.h); a
 * CPU test sweeps both and requires bitwise-identical results.
 *
 * Algorithm: Cody-Waite reduction by pi/2 with a three-part constant, then the
 * published fdlibm minimax coefficients (__kernel_sin / __kernel_cos, |r| <= pi/4),
 * evaluated in Estrin form.
 * Every operation is an IEEE-754 double op or an explicit fma(), so the result
 * is bit-identical on any IEEE host and on gfx950 (v_fma_f64 is correctly
 * rounded).  Compile with -ffp-contract=off.
 */
#ifndef OR_SINCOS_H
#define OR_SINCOS_H
#include <math.h>

static inline void or_sincos_kernel(double r, double *s, double *c)
{
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    /* Estrin evaluation (3 fma levels instead of 5): the Costas recurrence
     * waits on this chain every symbol */
    double z = r * r;
    double zz = z * z;
    /* sin: r + r^3 (S1 + z S2 + z^2 S3 + z^3 S4 + z^4 S5 + z^5 S6) */
    double sa = fma(z, S2, S1), sb = fma(z, S4, S3), sc = fma(z, S6, S5);
    double ps = fma(zz, fma(zz, sc, sb), sa);
    double v = z * r;
    *s = fma(v, ps, r);
    /* cos: 1 - z/2 + z^2 (C1 + z C2 + ... + z^5 C6), fdlibm tail correction */
    double ca = fma(z, C2, C1), cb = fma(z, C4, C3), cc = fma(z, C6, C5);
    double pc = fma(zz, fma(zz, cc, cb), ca);
    double hz = 0.5 * z;
    double w = 1.0 - hz;
    *c = w + (((1.0 - w) - hz) + zz * pc);
}

static inline void or_sincos(double x, double *s, double *c)
{
    /* straight-line on the common path: the GPU Costas loop is issue-bound and
     * every branch or select costs issue slots.  NaN propagates through the
     * arithmetic; |x| > 1e6 (and +-Inf -> NaN) take a pre-reduction branch
     * that the Costas loop never reaches (theta is wrapped to [-pi, pi]). */
    const double INVPIO2 = 6.36619772367581382433e-01;
    const double P1 = 1.57079632679489655800e+00;  /* pi/2 rounded to double */
    const double P2 = 6.12323399573676603587e-17;  /* next 53 bits */
    const double P3 = -1.49738490485916983e-33;    /* next bits */
    if (__builtin_expect(fabs(x) > 1.0e6, 0)) x = fmod(x, 6.28318530717958647693);
    const double k = rint(x * INVPIO2);
    double r = fma(-k, P1, x);
    r = fma(-k, P2, r);
    r = fma(-k, P3, r);
    double ks, kc;
    or_sincos_kernel(r, &ks, &kc);
    /* quadrant = low bits of the integer k (|k| < 2^20): k + 1.5*2^52 puts
     * them in the low mantissa bits; well defined for NaN too (result is NaN) */
    union { double d; unsigned long long u; } kb;
    kb.d = k + 6755399441055744.0;
    const unsigned q = (unsigned)(kb.u & 3u);
    /* q: 0 -> (s, c), 1 -> (c, -s), 2 -> (-s, -c), 3 -> (-c, s) */
    union { double d; unsigned long long u; } sv, cv;
    sv.d = (q & 1u) ? kc : ks;
    cv.d = (q & 1u) ? ks : kc;
    sv.u ^= (unsigned long long)(q & 2u) << 62;
    cv.u ^= (unsigned long long)((q + 1u) & 2u) << 62;
    *s = sv.d;
    *c = cv.d;
}

static inline void or_sincosf(float x, float *s, float *c)
{
    double sd, cd;
    or_sincos((double)x, &sd, &cd);
    *s = (float)sd;
    *c = (float)cd;
}
#endif
