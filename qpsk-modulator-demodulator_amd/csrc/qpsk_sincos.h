/*
 * qpsk_sincos.h -- PRODUCT copy of the portable double/float sin+cos used as the
 * deterministic stand-in for .NET Math.Cos/Math.Sin (CostasLoopQpsk.cs:69-70)
 * and MathF.Cos/MathF.Sin (Band-Edge Filter.cs:108-109).
 *
 * Host + device.  The oracle keeps its own copy (oracle/or_sincos.h); a CPU
 * test sweeps both and requires bitwise-identical results, and the GPU parity
 * tests require the GPU Costas/FLL outputs to equal the oracle's bit for bit.
 *
 * Algorithm: Cody-Waite reduction by pi/2 with a three-part constant, then the
 * published fdlibm minimax kernels (__kernel_sin / __kernel_cos, |r| <= pi/4).
 * Every operation is an IEEE-754 double op or an explicit fma(), so the result
 * is bit-identical on any IEEE host and on gfx950 (v_fma_f64 is correctly
 * rounded).  Compile with -ffp-contract=off.
 */
#ifndef QPSK_SINCOS_H
#define QPSK_SINCOS_H
#include <math.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define QPSK_HD __host__ __device__
#else
#define QPSK_HD
#endif

QPSK_HD static inline void qpsk_sincos_kernel(double r, double *s, double *c)
{
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = r * r;
    /* sin */
    double ps = fma(z, S6, S5);
    ps = fma(z, ps, S4);
    ps = fma(z, ps, S3);
    ps = fma(z, ps, S2);
    ps = fma(z, ps, S1);
    double v = z * r;
    *s = fma(v, ps, r);
    /* cos */
    double pc = fma(z, C6, C5);
    pc = fma(z, pc, C4);
    pc = fma(z, pc, C3);
    pc = fma(z, pc, C2);
    pc = fma(z, pc, C1);
    double hz = 0.5 * z;
    double w = 1.0 - hz;
    double zz = z * z;
    *c = w + (((1.0 - w) - hz) + zz * pc);
}

QPSK_HD static inline void qpsk_sincos(double x, double *s, double *c)
{
    const double INVPIO2 = 6.36619772367581382433e-01;
    const double P1 = 1.57079632679489655800e+00;  /* pi/2 rounded to double */
    const double P2 = 6.12323399573676603587e-17;  /* next 53 bits */
    const double P3 = -1.49738490485916983e-33;    /* next bits */
    if (!(fabs(x) <= 1.0e300)) { *s = x - x; *c = x - x; return; } /* NaN / Inf -> NaN */
    if (fabs(x) > 1.0e6) x = fmod(x, 6.28318530717958647693);
    double k = rint(x * INVPIO2);
    double r = fma(-k, P1, x);
    r = fma(-k, P2, r);
    r = fma(-k, P3, r);
    double ks, kc;
    qpsk_sincos_kernel(r, &ks, &kc);
    int q = ((int)k) & 3;
    switch (q) {
    case 0: *s = ks; *c = kc; break;
    case 1: *s = kc; *c = -ks; break;
    case 2: *s = -ks; *c = -kc; break;
    default: *s = -kc; *c = ks; break;
    }
}

QPSK_HD static inline void qpsk_sincosf(float x, float *s, float *c)
{
    double sd, cd;
    qpsk_sincos((double)x, &sd, &cd);
    *s = (float)sd;
    *c = (float)cd;
}
#endif
