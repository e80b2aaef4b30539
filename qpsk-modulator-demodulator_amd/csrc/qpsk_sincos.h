/*
 * qpsk_sincos.h -- PRODUCT copy of the portable double/float sin+cos used as the
 * deterministic stand-in for .NET Math.Cos/Math.Sin (CostasLoopQpsk.cs:69-70)
 * (the float MathF.Cos/MathF.Sin of the FLL are glibc's, qpsk_sincosf.h).
 *
 * Host + device.  The oracle keeps its own copy (oracle/or_sincos.h); a CPU
 * test sweeps both and requires bitwise-identical results, and the GPU parity
 * tests require the GPU Costas/FLL outputs to equal the oracle's bit for bit.
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
#ifndef QPSK_SINCOS_H
#define QPSK_SINCOS_H
#include <math.h>
#include "qpsk_sincos_table.h"
#include "qpsk_sincosf.h"
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define QPSK_HD __host__ __device__
#else
#define QPSK_HD
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define QPSK_SINCOS_SCHED_BARRIER() __builtin_amdgcn_sched_barrier(0)
#else
#define QPSK_SINCOS_SCHED_BARRIER() ((void)0)
#endif

/* [2k] = sin(k pi/256), [2k+1] = cos(k pi/256), k < 512: correctly rounded
 * double + float tail (tools/gen_sincos_table.py) */
static const double qpsk_sincos_table_host[1024] = { QPSK_SINCOS_TAB_VALUES_HI };
static const double qpsk_sincos_table_host_lo[1024] = { QPSK_SINCOS_TAB_VALUES_LO };
#if defined(__HIPCC__)
/* device copy; kernels stage it into LDS once per workgroup */
static __device__ const double qpsk_sincos_table_dev[1024] = { QPSK_SINCOS_TAB_VALUES_HI };
static __device__ const double qpsk_sincos_table_dev_lo[1024] = { QPSK_SINCOS_TAB_VALUES_LO };
#endif

/* argument the table reduction accepts: |x| <= 2^40 (or NaN).  Up to there
 * k = rint(x*256/pi) < 2^49 and x - k*P1 is a multiple of 2^-59 below 2^-6
 * (so the first fma is exact); the second part leaves k*(pi/256 - P1 - P2),
 * below 2^-106 for |x| <= 8 (the Costas phase in lock) and 2^-69 at 2^40.
 * Larger |x| and +-Inf are pre-reduced with fmod (Inf -> NaN).  The Costas
 * loop's theta leaves [-pi, pi] only once its freq passes pi (a QPSK false
 * lock at a multiple of pi/2 per symbol): theta then grows by ~freq per
 * symbol, which a sustained run reaches within a few calls. */
QPSK_HD static inline double qpsk_sincos_arg(double x)
{
    return fabs(x) > 0x1p40 ? fmod(x, 6.28318530717958647693) : x;
}

/* the core's constants; a caller may hold them in registers (device loops pin
 * them in VGPRs so no iteration rebuilds 64-bit constants) */
typedef struct {
    double INV, SH, P1, P2, S3, S5, C4, C6;
} qpsk_sincos_consts;
#define QPSK_SINCOS_CONSTS_INIT                                                    \
    {                                                                              \
        0x1.45f306dc9c883p+6,      /* 256/pi */                                    \
        0x1.8p+52,                 /* 1.5*2^52: ulp 1 */                           \
        0x1.921fb54442d18p-7,      /* pi/256 rounded to double */                  \
        0x1.1a62633145c07p-61,     /* next 53 bits */                              \
        -0x1.5555555555555p-3, 0x1.1111111111111p-7,   /* -1/6, 1/120 */           \
        0x1.5555555555555p-5, -0x1.6c16c16c16c17p-10   /* 1/24, -1/720 */          \
    }

/* the table row of x and the shifted multiple (first half of the core) */
typedef struct {
    double x, kb;
    double ts, tc, ls, lc;
} qpsk_sincos_row;

QPSK_HD static inline qpsk_sincos_row qpsk_sincos_tab_load(double x, const double *tab, const double *lo,
                                                           const qpsk_sincos_consts *K)
{
    /* kb = fma(x, 256/pi, 1.5*2^52) rounds the exact product to an integer
     * (ties to even), so k = kb - 1.5*2^52 = rint(x*256/pi) exactly
     * (|x| <= 2^40) and the low mantissa bits of kb are k mod 512 in two's
     * complement: the table index without a separate rint */
    union { double d; unsigned long long u; } kb;
    kb.d = fma(x, K->INV, K->SH);
    const unsigned i = (unsigned)(kb.u & 511u) * 2u;
    qpsk_sincos_row R;
    R.x = x;
    R.kb = kb.d;
    R.ts = tab[i];
    R.tc = tab[i + 1];
    R.ls = lo[i];
    R.lc = lo[i + 1];
    return R;
}

/* the second half: reduction, polynomials, angle addition */
QPSK_HD static inline void qpsk_sincos_tab_eval(const qpsk_sincos_row *R, const qpsk_sincos_consts *K, double *s,
                                                double *c)
{
    const double k = R->kb - K->SH;
    double r = fma(-k, K->P1, R->x);               /* Cody-Waite: |r| <= pi/512 */
    r = fma(-k, K->P2, r);
    /* sin r = r + r^3(-1/6 + r^2/120), cos r - 1 = r^2(-1/2 + r^2/24 - r^4/720):
     * truncation < 1e-19 relative for |r| <= pi/512 */
    const double z = r * r;
    const double r3p = (r * z) * fma(z, K->S5, K->S3);          /* sin r - r */
    const double cm = z * fma(z, fma(z, K->C6, K->C4), -0.5);   /* cos r - 1 */
    /* angle addition, small terms first: sin x = ts + [tc r + (tc r3p + ts cm + ls)],
     * one significant rounding in the bracket and one in the final add: <= 1 ulp */
    *s = R->ts + fma(R->tc, r, fma(R->tc, r3p, fma(R->ts, cm, R->ls)));
    *c = R->tc + fma(-R->ts, r, fma(-R->ts, r3p, fma(R->tc, cm, R->lc)));
}

/* both halves; on the GPU the row's loads go out first: the scheduler may not
 * move the reduction or the polynomials ahead of them (a GPU caller with work
 * of its own for the LDS round trip calls the halves itself) */
QPSK_HD static inline void qpsk_sincos_tab_core_k(double x, const double *tab, const double *lo,
                                             const qpsk_sincos_consts *K, double *s, double *c)
{
    const qpsk_sincos_row R = qpsk_sincos_tab_load(x, tab, lo, K);
    QPSK_SINCOS_SCHED_BARRIER();
    qpsk_sincos_tab_eval(&R, K, s, c);
}

/* sin and cos of x, |x| <= 2^40 or NaN, given the 512-entry table (any address
 * space: the GPU kernels pass a copy staged in LDS).  Straight-line: the GPU
 * Costas loop is issue-bound and every instruction costs issue slots.  NaN
 * propagates (any table index gives NaN). */
QPSK_HD static inline void qpsk_sincos_tab_core(double x, const double *tab, const double *lo,
                                           double *s, double *c)
{
    const qpsk_sincos_consts K = QPSK_SINCOS_CONSTS_INIT;
    qpsk_sincos_tab_core_k(x, tab, lo, &K, s, c);
}

/* any x: the pre-reduction branch, then the table reduction */
QPSK_HD static inline void qpsk_sincos_tab(double x, const double *tab, const double *lo, double *s,
                                      double *c)
{
    if (__builtin_expect(fabs(x) > 0x1p40, 0)) x = qpsk_sincos_arg(x);
    qpsk_sincos_tab_core(x, tab, lo, s, c);
}

static inline void qpsk_sincos(double x, double *s, double *c)
{
    qpsk_sincos_tab(x, qpsk_sincos_table_host, qpsk_sincos_table_host_lo, s, c);
}

/* float sin/cos (MathF.Sin/Cos of the FLL phase): glibc's sinf/cosf restated,
 * qpsk_sincosf.h */
static inline void qpsk_sincosf(float x, float *s, float *c)
{
    qpsk_sincosf_glibc(x, s, c);
}
#endif
