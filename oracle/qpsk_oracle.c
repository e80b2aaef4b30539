/*
 * qpsk_oracle.c -- CPU restatement of the reference C# QPSK demodulation chain.
 *
 * TEST INFRASTRUCTURE ONLY (see qpsk_oracle.h).  Nothing in the product
 * library links or calls this file.  Parity with the C# itself is UNPINNED
 * (no .NET runtime here, no golden vectors in the reference): see
 * DESIGN.md "Oracle".
 *
 * Numeric rules followed:
 *  - no FMA contraction anywhere (build with -ffp-contract=off); .NET RyuJIT
 *    never contracts a*b+c;
 *  - Vector<float>.Count lane order for every FIR dot product
 *    (FIRFilter.cs:156-192), lanes = 8 on AVX2 x64;
 *  - Math.Round is round-half-even (RRC-filter.cs:24,26) -> nearbyint;
 *  - float/double boundaries exactly as the C# casts;
 *  - MathF.IEEERemainder -> remainderf.
 */
#define _GNU_SOURCE
#include "qpsk_oracle.h"
#include "or_sincos.h"
#include <ctype.h>
#include <immintrin.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define OR_PI 3.14159265358979311600     /* Math.PI */
#define OR_TWO_PI_D (2.0 * OR_PI)         /* CostasLoopQpsk.cs:89 */
#define OR_PI_F 3.14159274101257324219f  /* MathF.PI */

/* Math.Pow goes to the platform libm; keep gcc from folding pow(x, 2.0) into
 * x*x (glibc pow(x, 2.0) is not always the correctly rounded x*x). */
static double (*volatile or_pow)(double, double) = pow;
/* Math.Sin / Math.Cos (and the MathF pair) are separate libm calls in .NET;
 * gcc would merge a sin and a cos of one argument into one sincos() call
 * (its cse_sincos pass, no -ffast-math needed), and glibc's sincos is not
 * bit-identical to sin (0.855 <= |x| < 2.426 reduces pi/2 - |x| differently).
 * Calls through volatile pointers keep them separate, as .NET makes them. */
static double (*volatile or_libm_sin)(double) = sin;
static double (*volatile or_libm_cos)(double) = cos;
static float (*volatile or_libm_sinf)(float) = sinf;
static float (*volatile or_libm_cosf)(float) = cosf;

static void trig_d(int mode, double x, double *s, double *c)
{
    if (mode == OR_TRIG_PORTABLE) {
        or_sincos(x, s, c);
    } else {
        *c = or_libm_cos(x);                 /* CostasLoopQpsk.cs:69 */
        *s = or_libm_sin(x);                 /* :70 */
    }
}

static void trig_f(int mode, float x, float *s, float *c)
{
    if (mode == OR_TRIG_PORTABLE) {
        or_sincosf(x, s, c);
    } else {
        *c = or_libm_cosf(x);
        *s = or_libm_sinf(x);
    }
}

/* ------------------------------------------------------------------------ */
/* RRC-filter.cs:16-75  generateCoefficents                                  */
/* ------------------------------------------------------------------------ */
int or_rrc_taps(double span_symbols, double beta, int sample_rate, int symbol_rate, double *out,
                int cap)
{
    double sps_exact = (double)sample_rate / symbol_rate;      /* :24 */
    int sps = (int)nearbyint(sps_exact);                        /* Math.Round, half-even */
    int span_int = (int)nearbyint(span_symbols);                /* :26 */
    int taps = span_int * sps + 1;                              /* :27 */
    if (taps <= 0 || taps > cap) return -taps;
    int mid = (taps - 1) / 2;
    const double pi = OR_PI;
    const double eps = 1e-8;
    for (int n = 0; n < taps; n++) {
        double t = (n - mid) / (double)sps;                    /* :38 */
        double val;
        if (fabs(t) < eps) {
            val = 1.0 + beta * (4.0 / pi - 1.0);                /* :44 */
        } else if (fabs(fabs(t) - 1.0 / (4.0 * beta)) < eps) {
            val = (beta / sqrt(2.0)) *
                  ((1.0 + 2.0 / pi) * or_libm_sin(pi / (4.0 * beta)) +
                   (1.0 - 2.0 / pi) * or_libm_cos(pi / (4.0 * beta))); /* :49-51 */
        } else {
            double num = or_libm_sin(pi * t * (1.0 - beta)) + 4.0 * beta * t * or_libm_cos(pi * t * (1.0 + beta));
            double den = pi * t * (1.0 - or_pow(4.0 * beta * t, 2.0));
            val = num / den;                                    /* :56-59 */
        }
        out[n] = val;
    }
    double energy = 0.0;                                        /* :65-72 */
    for (int i = 0; i < taps; i++) energy += out[i] * out[i];
    double norm = sqrt(energy);
    for (int i = 0; i < taps; i++) out[i] /= norm;
    return taps;
}

/* ------------------------------------------------------------------------ */
/* FIRFilter.cs:8-232  ComplexFIRFilter (streaming, Vector<float> order)     */
/* ------------------------------------------------------------------------ */
struct or_cfir {
    int n;          /* _nTaps */
    int lanes;      /* Vector<float>.Count; <=1 -> non-accelerated path */
    int pos;        /* _pos */
    float *tir, *tqr;   /* _tapsIRev, _tapsQRev */
    float *di, *dq;     /* _delayI2N, _delayQ2N */
};

or_cfir *or_cfir_new(const float *taps_iq, int n_floats, int lanes)
{
    if ((n_floats & 1) || n_floats == 0) return NULL;           /* :32-33 */
    or_cfir *f = (or_cfir *)calloc(1, sizeof(*f));
    f->n = n_floats >> 1;
    f->lanes = lanes;
    f->tir = (float *)calloc(f->n, sizeof(float));
    f->tqr = (float *)calloc(f->n, sizeof(float));
    for (int k = 0; k < f->n; k++) {                            /* :43-48 */
        int src = (f->n - 1 - k) << 1;
        f->tir[k] = taps_iq[src];
        f->tqr[k] = taps_iq[src + 1];
    }
    f->di = (float *)calloc(2 * f->n, sizeof(float));
    f->dq = (float *)calloc(2 * f->n, sizeof(float));
    f->pos = 0;
    return f;
}

void or_cfir_free(or_cfir *f)
{
    if (!f) return;
    free(f->tir); free(f->tqr); free(f->di); free(f->dq);
    free(f);
}

/* FIRFilter.cs:144-211 ComplexDotWindow */
static void cfir_dot(const or_cfir *f, int start, float *out_i, float *out_q)
{
    float acc_i = 0.0f, acc_q = 0.0f;
    const int n = f->n;
    const float *xi = f->di + start, *xq = f->dq + start;
    const float *hi = f->tir, *hq = f->tqr;
    if (f->lanes == 8) {
        /* Vector<float> on AVX2 x64 = one ymm register per accumulator: the
         * same per-lane IEEE ops as the generic branch, issued as AVX2 */
        const int nvec = n - (n % 8);
        __m256 vi = _mm256_setzero_ps(), vq = _mm256_setzero_ps();
        for (int i = 0; i < nvec; i += 8) {
            __m256 xi8 = _mm256_loadu_ps(xi + i), xq8 = _mm256_loadu_ps(xq + i);
            __m256 hi8 = _mm256_loadu_ps(hi + i), hq8 = _mm256_loadu_ps(hq + i);
            vi = _mm256_add_ps(vi, _mm256_sub_ps(_mm256_mul_ps(hi8, xi8), _mm256_mul_ps(hq8, xq8)));
            vq = _mm256_add_ps(vq, _mm256_add_ps(_mm256_mul_ps(hi8, xq8), _mm256_mul_ps(hq8, xi8)));
        }
        float va_i[8], va_q[8];
        _mm256_storeu_ps(va_i, vi);
        _mm256_storeu_ps(va_q, vq);
        for (int l = 0; l < 8; l++) {
            acc_i += va_i[l];
            acc_q += va_q[l];
        }
        for (int i = nvec; i < n; i++) {
            acc_i += (hi[i] * xi[i]) - (hq[i] * xq[i]);
            acc_q += (hi[i] * xq[i]) + (hq[i] * xi[i]);
        }
    } else if (f->lanes > 1) {
        const int w = f->lanes;
        const int nvec = n - (n % w);
        float va_i[64], va_q[64];
        for (int l = 0; l < w; l++) { va_i[l] = 0.0f; va_q[l] = 0.0f; }
        for (int i = 0; i < nvec; i += w) {                     /* :165-174 */
            for (int l = 0; l < w; l++) {
                float a = hi[i + l] * xi[i + l];
                float b = hq[i + l] * xq[i + l];
                float c = hi[i + l] * xq[i + l];
                float d = hq[i + l] * xi[i + l];
                va_i[l] = va_i[l] + (a - b);
                va_q[l] = va_q[l] + (c + d);
            }
        }
        for (int l = 0; l < w; l++) {                           /* :176-180 */
            acc_i += va_i[l];
            acc_q += va_q[l];
        }
        for (int i = nvec; i < n; i++) {                        /* :183-192 */
            acc_i += (hi[i] * xi[i]) - (hq[i] * xq[i]);
            acc_q += (hi[i] * xq[i]) + (hq[i] * xi[i]);
        }
    } else {
        for (int i = 0; i < n; i++) {                           /* :197-206 */
            acc_i += (hi[i] * xi[i]) - (hq[i] * xq[i]);
            acc_q += (hi[i] * xq[i]) + (hq[i] * xi[i]);
        }
    }
    *out_i = acc_i;
    *out_q = acc_q;
}

/* FIRFilter.cs:59-77 Filter(sample) */
static inline void cfir_sample(or_cfir *f, float in_i, float in_q, float *out_i, float *out_q)
{
    int p = f->pos;
    int pn = p + f->n;
    f->di[p] = in_i; f->dq[p] = in_q;
    f->di[pn] = in_i; f->dq[pn] = in_q;
    int start = p + 1;
    if (start >= f->n) start -= f->n;
    cfir_dot(f, start, out_i, out_q);
    p++;
    if (p == f->n) p = 0;
    f->pos = p;
}

/* FIRFilter.cs:80-91 Filter(span) */
void or_cfir_filter(or_cfir *f, const float *in_iq, float *out_iq, long n_complex)
{
    for (long s = 0; s < n_complex; s++) {
        float yi, yq;
        cfir_sample(f, in_iq[2 * s], in_iq[2 * s + 1], &yi, &yq);
        out_iq[2 * s] = yi;
        out_iq[2 * s + 1] = yq;
    }
}

/* ------------------------------------------------------------------------ */
/* MuellerMuller.cs:17-249                                                   */
/* ------------------------------------------------------------------------ */
struct or_mm {
    double sps, kp, ki;
    int base;            /* baseIndex */
    double mu;
    double integ;        /* ncoIntegral */
    float psi, psq;      /* prevSample */
    float pdi, pdq;      /* prevDecision */
    int has_prev;
    float *buf;          /* _bufIQ */
    long cap;            /* floats */
    long start, count;   /* complex samples */
};

or_mm *or_mm_new(double sps, double kp, double ki)
{
    or_mm *m = (or_mm *)calloc(1, sizeof(*m));
    m->sps = sps; m->kp = kp; m->ki = ki;
    m->base = 1;                                                /* :44 */
    m->mu = 0.0;
    m->integ = 0.0;
    m->has_prev = 0;
    m->cap = 4096;
    m->buf = (float *)calloc(m->cap, sizeof(float));
    return m;
}

void or_mm_free(or_mm *m)
{
    if (!m) return;
    free(m->buf);
    free(m);
}

/* :200-249 Append / EnsureCapacityForAppend / Compact (numerically inert) */
static void mm_append(or_mm *m, const float *in, long n_floats)
{
    long inc = n_floats >> 1;
    if (inc == 0) return;
    if (m->start > 0) {
        memmove(m->buf, m->buf + 2 * m->start, (size_t)(2 * m->count) * sizeof(float));
        m->start = 0;
    }
    long need = 2 * (m->count + inc);
    if (need > m->cap) {
        long nl = m->cap;
        while (nl < need) nl <<= 1;
        m->buf = (float *)realloc(m->buf, (size_t)nl * sizeof(float));
        m->cap = nl;
    }
    memcpy(m->buf + 2 * m->count, in, (size_t)(2 * inc) * sizeof(float));
    m->count += inc;
}

/* :160-190 CubicLagrange4 */
static inline void mm_lagrange(const or_mm *m, long n, double mu, float *oi, float *oq)
{
    const float *b = m->buf + 2 * (m->start + n - 1);
    float xm1i = b[0], xm1q = b[1], x0i = b[2], x0q = b[3];
    float x1i = b[4], x1q = b[5], x2i = b[6], x2q = b[7];
    float t = (float)mu;
    float tm1 = t - 1.0f;
    float tm2 = t - 2.0f;
    float tp1 = t + 1.0f;
    float cm1 = -(t * tm1 * tm2) * (1.0f / 6.0f);
    float c0 = (tp1 * tm1 * tm2) * (1.0f / 2.0f);
    float c1 = -(tp1 * t * tm2) * (1.0f / 2.0f);
    float c2 = (tp1 * t * tm1) * (1.0f / 6.0f);
    *oi = cm1 * xm1i + c0 * x0i + c1 * x1i + c2 * x2i;
    *oq = cm1 * xm1q + c0 * x0q + c1 * x1q + c2 * x2q;
}

/* (int)d in .NET 9: saturating, NaN -> 0 (x64 conversions were made
 * saturating in .NET 9; C leaves NaN and out-of-range undefined) */
static int or_dotnet_int(double d)
{
    if (d != d) return 0;
    if (d >= 2147483647.0) return 2147483647;
    if (d <= -2147483648.0) return (int)-2147483647 - 1;
    return (int)d;
}

/* :52-136 Process(span).  Returns the symbol count, -1 for an odd length, or
 * OR_ERR_INDEX where the C# indexer would throw IndexOutOfRangeException: a
 * NaN timing pins baseIndex at (int)Math.Floor(NaN) = 0, and CubicLagrange4
 * then reads _bufIQ[(_bufStart - 1) * 2] (:164), out of range while
 * _bufStart == 0. */
long or_mm_process(or_mm *m, const float *in_iq, long n_floats, float *out_iq, long out_floats)
{
    if (n_floats & 1) return -1;
    mm_append(m, in_iq, n_floats);
    long out_sym = 0;
    while (m->base + 2 < m->count) {
        if (m->start + m->base - 1 < 0) return OR_ERR_INDEX;
        float ci, cq;
        mm_lagrange(m, m->base, m->mu, &ci, &cq);
        float di = (ci >= 0.0f) ? 1.0f : -1.0f;                /* :194-198 */
        float dq = (cq >= 0.0f) ? 1.0f : -1.0f;
        double adv;
        if (m->has_prev) {
            double t1 = (double)m->pdi * ci + (double)m->pdq * cq;  /* :78 */
            double t2 = (double)di * m->psi + (double)dq * m->psq;  /* :79 */
            double e = t1 - t2;
            m->integ += m->ki * e;                                   /* :83 */
            double corr = m->kp * e + m->integ;
            const double max_step = 0.1;
            if (corr > max_step) corr = max_step;
            if (corr < -max_step) corr = -max_step;
            adv = m->sps + corr;
        } else {
            m->has_prev = 1;
            adv = m->sps;
        }
        long o = out_sym << 1;
        if (o + 1 >= out_floats) break;                              /* :101-102 */
        out_iq[o] = ci;
        out_iq[o + 1] = cq;
        out_sym++;
        m->psi = ci; m->psq = cq;
        m->pdi = di; m->pdq = dq;
        double nt = m->base + m->mu + adv;                           /* :113 */
        m->base = or_dotnet_int(floor(nt));
        m->mu = nt - m->base;
        if (m->base + 1 >= m->count) break;
    }
    long a = m->base - 1; if (a < 0) a = 0;                          /* :123 */
    long b = m->count - 3; if (b < 0) b = 0;
    long consumed = a < b ? a : b;
    if (consumed > 0) {
        m->start += consumed;
        m->count -= consumed;
        m->base -= (int)consumed;
    }
    return out_sym;
}

/* ------------------------------------------------------------------------ */
/* IQ Balancer.cs:10-26                                                      */
/* ------------------------------------------------------------------------ */
void or_iqb_process(or_iqb *b, const float *in_iq, float *out_iq, long n_floats, int literal)
{
    const float ratio = 1e-05f;                                   /* :14 */
    const long end = literal ? n_floats / 2 : n_floats;           /* :17 (i < IN.Length/2) */
    for (long i = 0; i < end; i += 2) {
        b->avg_re = ratio * (in_iq[i] - b->avg_re) + b->avg_re;   /* :19-20 */
        b->avg_im = ratio * (in_iq[i + 1] - b->avg_im) + b->avg_im;
        out_iq[i] = in_iq[i] - b->avg_re;                         /* :21-22 */
        out_iq[i + 1] = in_iq[i + 1] - b->avg_im;
    }
}

/* ------------------------------------------------------------------------ */
/* CostasLoopQpsk.cs:19-130                                                  */
/* ------------------------------------------------------------------------ */
struct or_costas {
    double alpha, beta, theta, freq;
    int trig;
};

or_costas *or_costas_new(double sample_rate, double loop_bw_hz, double damping, int trig_mode)
{
    or_costas *c = (or_costas *)calloc(1, sizeof(*c));
    double bw = 2.0 * OR_PI * loop_bw_hz / sample_rate;          /* :39 */
    double d = 1.0 + 2.0 * damping * bw + bw * bw;                /* :42 */
    c->alpha = (4.0 * damping * bw) / d;
    c->beta = (4.0 * bw * bw) / d;
    c->theta = 0.0;
    c->freq = 0.0;
    c->trig = trig_mode;
    return c;
}

void or_costas_free(or_costas *c) { free(c); }

void or_costas_state(const or_costas *c, double *theta, double *freq)
{
    *theta = c->theta;
    *freq = c->freq;
}

/* :63-92 */
void or_costas_process(or_costas *c, float in_i, float in_q, float *out_i, float *out_q)
{
    double cs, sn;
    trig_d(c->trig, c->theta, &sn, &cs);
    double mi = (double)in_i * cs + (double)in_q * sn;
    double mq = (double)in_q * cs - (double)in_i * sn;
    float oi = (float)mi, oq = (float)mq;
    *out_i = oi;
    *out_q = oq;
    float ei = (oi >= 0.0f) ? 1.0f : -1.0f;                       /* :52-56 */
    float eq = (oq >= 0.0f) ? 1.0f : -1.0f;
    double pe = (double)ei * mq - (double)eq * mi;                 /* :82 */
    c->freq += c->beta * pe;
    c->theta += c->freq + c->alpha * pe;
    if (c->theta > OR_PI) c->theta -= OR_TWO_PI_D;
    else if (c->theta < -OR_PI) c->theta += OR_TWO_PI_D;
}

/* ------------------------------------------------------------------------ */
/* Band-Edge Filter.cs:14-203  FLLBandEdgeFilter                             */
/* ------------------------------------------------------------------------ */
struct or_fll {
    float sps, rolloff, bandwidth;
    int filter_size;
    float phase, freq;
    float alpha, beta, max_freq, min_freq;
    float *lower_iq, *upper_iq;
    or_cfir *f_lower, *f_upper;
    int trig;
};

static float fll_sinc(float x)                                    /* :197-202 */
{
    if (x == 0.0f) return 1.0f;
    float arg = OR_PI_F * x;
    return or_libm_sinf(arg) / arg;
}

or_fll *or_fll_new(float sps, float rolloff, int filter_size, float bandwidth, int lanes,
                   int trig_mode)
{
    if (sps <= 0.0f) return NULL;                                  /* :42-45 */
    if (rolloff < 0 || rolloff > 1.0f) return NULL;
    if (filter_size <= 0) return NULL;
    if (bandwidth <= 0.0f) return NULL;
    const float TWO_PI = 2.0f * OR_PI_F;
    or_fll *f = (or_fll *)calloc(1, sizeof(*f));
    f->sps = sps; f->rolloff = rolloff; f->filter_size = filter_size; f->bandwidth = bandwidth;
    f->phase = 0.0f; f->freq = 0.0f;
    f->alpha = 0.0f;
    f->beta = 4.0f * bandwidth / sps;                             /* :56 */
    f->max_freq = TWO_PI * (2.0f / sps);
    f->min_freq = -f->max_freq;
    f->trig = trig_mode;
    /* DesignFilter :132-183 (host-side taps: libm sinf/cosf in both modes) */
    int nt = filter_size;
    int mid = (nt - 1) / 2;
    float *bb = (float *)calloc(nt, sizeof(float));
    float sum = 0.0f;
    for (int i = 0; i < nt; i++) {
        float k = (float)(i - mid) / (2.0f * sps);
        float pos = rolloff * k;
        float tap = fll_sinc(pos - 0.5f) + fll_sinc(pos + 0.5f);
        sum += tap;
        bb[i] = tap;
    }
    for (int i = 0; i < nt; i++) bb[i] /= sum;
    f->lower_iq = (float *)calloc(2 * nt, sizeof(float));
    f->upper_iq = (float *)calloc(2 * nt, sizeof(float));
    for (int i = 0; i < nt; i++) {
        float k = (float)(i - mid) / (2.0f * sps);
        float angle = -TWO_PI * (1.0f + rolloff) * k;
        float wc = or_libm_cosf(angle);
        float ws = or_libm_sinf(angle);
        float li = bb[i] * wc;
        float lq = bb[i] * ws;
        f->lower_iq[2 * i] = li; f->lower_iq[2 * i + 1] = lq;
        f->upper_iq[2 * i] = li; f->upper_iq[2 * i + 1] = -lq;
    }
    free(bb);
    f->f_lower = or_cfir_new(f->lower_iq, 2 * nt, lanes);
    f->f_upper = or_cfir_new(f->upper_iq, 2 * nt, lanes);
    return f;
}

void or_fll_free(or_fll *f)
{
    if (!f) return;
    or_cfir_free(f->f_lower); or_cfir_free(f->f_upper);
    free(f->lower_iq); free(f->upper_iq);
    free(f);
}

int or_fll_taps(const or_fll *f, float *lower_iq, float *upper_iq, int cap_floats)
{
    int n = 2 * f->filter_size;
    if (n > cap_floats) return -n;
    memcpy(lower_iq, f->lower_iq, n * sizeof(float));
    memcpy(upper_iq, f->upper_iq, n * sizeof(float));
    return n;
}

void or_fll_state(const or_fll *f, float *phase, float *freq)
{
    *phase = f->phase;
    *freq = f->freq;
}

/* :102-129 Process(sample) */
static inline void fll_sample(or_fll *f, float in_i, float in_q, float *out_i, float *out_q)
{
    const float TWO_PI = 2.0f * OR_PI_F;
    float c, s;
    trig_f(f->trig, f->phase, &s, &c);
    float oi = in_i * c - in_q * s;
    float oq = in_i * s + in_q * c;
    *out_i = oi;
    *out_q = oq;
    float upi, upq, loi, loq;
    cfir_sample(f->f_upper, oi, oq, &upi, &upq);
    cfir_sample(f->f_lower, oi, oq, &loi, &loq);
    float pow_u = upi * upi + upq * upq;
    float pow_l = loi * loi + loq * loq;
    float err = pow_l - pow_u;
    f->freq += f->beta * err;
    f->phase += f->freq + f->alpha * err;
    if (f->phase > TWO_PI || f->phase < -TWO_PI)                  /* :185-189 */
        f->phase = remainderf(f->phase, TWO_PI);
    if (f->freq > f->max_freq) f->freq = f->max_freq;             /* :191-195 */
    else if (f->freq < f->min_freq) f->freq = f->min_freq;
}

void or_fll_process(or_fll *f, const float *in_iq, float *out_iq, long n_complex)
{
    for (long i = 0; i < n_complex; i++)
        fll_sample(f, in_iq[2 * i], in_iq[2 * i + 1], &out_iq[2 * i], &out_iq[2 * i + 1]);
}

/* ------------------------------------------------------------------------ */
/* HelperFunctions.cs:11-71 BitPacker                                        */
/* ------------------------------------------------------------------------ */
long or_bits_to_bytes(const char *bits, long n_bits, int bit_offset, uint8_t *out, long cap)
{
    if (bit_offset < 0 || bit_offset > 7) return -1;
    long usable = n_bits - bit_offset;
    if (usable < 8) return 0;
    long nb = usable / 8;
    if (nb > cap) return -2;
    long p = bit_offset;
    for (long i = 0; i < nb; i++) {
        uint8_t v = 0;
        for (int j = 0; j < 8; j++) {
            v = (uint8_t)(v << 1);
            if (bits[p++] == '1') v |= 1;
        }
        out[i] = v;
    }
    return nb;
}

long or_index_of(const uint8_t *hay, long n_hay, const uint8_t *needle, long n_needle)
{
    if (n_needle == 0) return 0;
    if (n_needle > n_hay) return -1;
    for (long i = 0; i <= n_hay - n_needle; i++)
        if (memcmp(hay + i, needle, (size_t)n_needle) == 0) return i;
    return -1;
}

/* ------------------------------------------------------------------------ */
/* QPSKDeModulator.cs                                                        */
/* ------------------------------------------------------------------------ */
struct or_demod {
    or_demod_cfg cfg;
    char *tsc;
    long tsc_len;
    or_cfir *rrc;
    or_fll *fll;
    or_mm *mm;
    or_costas *costas;
    double mm_sps, kp, ki;
    float *rrc_f32;
    int n_taps;
    float *tmp_fll, *tmp_rrc, *tmp_sym, *tmp_iqb;
    long tmp_cap;
    or_iqb iqb;
    /* differential decode state (:72-73) */
    int diff_have_prev;
    float prev_i, prev_q;
    /* framer state (:57-73) */
    uint8_t *ring;
    long ring_cap, rb_head, rb_count;
    int in_frame;
    char *carry;
    long carry_len;
    int locked_off;
    uint8_t pack_byte;
    int pack_bits;
    /* bit scratch */
    char *bits;
    long bits_cap;
};

void or_demod_cfg_default(or_demod_cfg *c, int sample_rate, int symbol_rate)
{
    memset(c, 0, sizeof(*c));
    c->sample_rate = sample_rate;
    c->symbol_rate = symbol_rate;
    c->rrc_alpha = 0.9f;                                          /* :14-18 */
    c->rrc_span = 6;
    c->symbol_sync_bw = 0.0001;
    c->costas_loop_bw = 120;
    c->cfo_loop_bw = (double)0.0001f;
    c->differential = 1;
    c->tsc = NULL;
    c->enable_fll = 0;
    c->lanes = 8;
    c->trig_mode = OR_TRIG_PORTABLE;
    c->ring_capacity = 300000000;
}

static int is_blank(const char *s)
{
    if (!s) return 1;
    for (; *s; s++)
        if (!isspace((unsigned char)*s)) return 0;
    return 1;
}

or_demod *or_demod_new(const or_demod_cfg *cfg, int *err)
{
    *err = 0;
    if (cfg->sample_rate <= 0 || cfg->symbol_rate <= 0) { *err = 2; return NULL; }
    or_demod *d = (or_demod *)calloc(1, sizeof(*d));
    d->cfg = *cfg;
    if (!is_blank(cfg->tsc)) {                                     /* :21 */
        d->tsc = strdup(cfg->tsc);
        d->tsc_len = (long)strlen(cfg->tsc);
    }
    /* :28-32 RRC (alpha float widened to double) */
    double taps[4096];
    int nt = or_rrc_taps((double)cfg->rrc_span, (double)cfg->rrc_alpha, cfg->sample_rate,
                         cfg->symbol_rate, taps, 4096);
    if (nt <= 0) { *err = 2; or_demod_free(d); return NULL; }
    d->n_taps = nt;
    d->rrc_f32 = (float *)calloc(nt, sizeof(float));
    float *tiq = (float *)calloc(2 * nt, sizeof(float));
    for (int i = 0; i < nt; i++) {                                 /* :278-288 */
        d->rrc_f32[i] = (float)taps[i];
        tiq[2 * i] = (float)taps[i];
        tiq[2 * i + 1] = 0.0f;
    }
    d->rrc = or_cfir_new(tiq, 2 * nt, cfg->lanes);
    free(tiq);
    /* :35 FLL (constructed even when unused; validation throws) */
    d->fll = or_fll_new((float)(cfg->sample_rate / cfg->symbol_rate), cfg->rrc_alpha, 40,
                        (float)cfg->cfo_loop_bw, cfg->lanes, cfg->trig_mode);
    if (!d->fll) { *err = 1; or_demod_free(d); return NULL; }
    /* :39-55 setupSymbolSync */
    {
        double sr = (double)cfg->sample_rate, yr = (double)cfg->symbol_rate;
        double zeta = 1.0 / sqrt(2.0);
        double bn = cfg->symbol_sync_bw;
        double wn = ((2.0 * OR_PI * bn) / (zeta + 0.25) / zeta);
        double denom = 1.0 + 2.0 * zeta * wn + wn * wn;
        d->kp = (4.0 * zeta * wn) / denom;
        d->ki = (4.0 * wn * wn) / denom;
        d->mm_sps = sr / yr;
        d->mm = or_mm_new(d->mm_sps, d->kp, d->ki);
    }
    /* :56 Costas(SymbolRate, SymbolRate / CostasLoopBandwith) */
    d->costas = or_costas_new((double)cfg->symbol_rate,
                              (double)cfg->symbol_rate / cfg->costas_loop_bw, 0.707,
                              cfg->trig_mode);
    d->ring_cap = cfg->ring_capacity > 0 ? cfg->ring_capacity : 300000000;
    d->locked_off = -1;
    return d;
}

void or_demod_free(or_demod *d)
{
    if (!d) return;
    free(d->tsc);
    or_cfir_free(d->rrc);
    or_fll_free(d->fll);
    or_mm_free(d->mm);
    or_costas_free(d->costas);
    free(d->rrc_f32);
    free(d->tmp_fll); free(d->tmp_rrc); free(d->tmp_sym); free(d->tmp_iqb);
    free(d->ring);
    free(d->carry);
    free(d->bits);
    free(d);
}

void or_demod_gains(const or_demod *d, double *mm_sps, double *kp, double *ki, double *c_alpha,
                    double *c_beta)
{
    *mm_sps = d->mm_sps; *kp = d->kp; *ki = d->ki;
    *c_alpha = d->costas->alpha; *c_beta = d->costas->beta;
}

int or_demod_rrc_f32(const or_demod *d, float *taps, int cap)
{
    if (d->n_taps > cap) return -d->n_taps;
    memcpy(taps, d->rrc_f32, d->n_taps * sizeof(float));
    return d->n_taps;
}

static void ensure_tmp(or_demod *d, long n_floats)               /* :290-302 */
{
    if (d->tmp_cap >= n_floats) return;
    long p = 1;
    while (p < n_floats) p <<= 1;
    d->tmp_fll = (float *)realloc(d->tmp_fll, (size_t)p * sizeof(float));
    d->tmp_rrc = (float *)realloc(d->tmp_rrc, (size_t)p * sizeof(float));
    d->tmp_sym = (float *)realloc(d->tmp_sym, (size_t)p * sizeof(float));
    d->tmp_iqb = (float *)realloc(d->tmp_iqb, (size_t)p * sizeof(float));
    d->tmp_cap = p;
}

/* :345-425 DeModulate, split so that tests can see the raw (pre-TSC) bits and
 * the symbols of the same call.  Returns the raw bit count. */
static long demod_core(or_demod *d, const float *iq, long n_floats, char *bits, long cap,
                       float *syms, long syms_cap, long *n_syms_out)
{
    ensure_tmp(d, n_floats);
    const float *src = iq;
    if (d->cfg.iq_balance) {                                      /* optional pre-stage */
        or_iqb_process(&d->iqb, src, d->tmp_iqb, n_floats, 0);
        src = d->tmp_iqb;
    }
    if (d->cfg.enable_fll) {                                      /* README.md:16 order */
        or_fll_process(d->fll, src, d->tmp_fll, n_floats >> 1);
        src = d->tmp_fll;
    }
    or_cfir_filter(d->rrc, src, d->tmp_rrc, n_floats >> 1);     /* :360 */
    long nsym = or_mm_process(d->mm, d->tmp_rrc, n_floats, d->tmp_sym, n_floats); /* :364 */
    if (nsym < 0) return nsym;                                    /* the C# call throws */
    long nb = 0;
    for (long k = 0; k < nsym; k++) {                             /* :372-408 */
        float si = d->tmp_sym[2 * k], sq = d->tmp_sym[2 * k + 1];
        float ri, rq;
        or_costas_process(d->costas, si, sq, &ri, &rq);
        if (syms && 2 * k + 1 < syms_cap) { syms[2 * k] = ri; syms[2 * k + 1] = rq; }
        float dec_i = (ri >= 0.0f) ? 1.0f : -1.0f;
        float dec_q = (rq >= 0.0f) ? 1.0f : -1.0f;
        char b0, b1;
        if (d->cfg.differential) {
            if (!d->diff_have_prev) {
                d->prev_i = dec_i; d->prev_q = dec_q;
                d->diff_have_prev = 1;
                continue;
            }
            float del_i = dec_i * d->prev_i + dec_q * d->prev_q;
            float del_q = dec_q * d->prev_i - dec_i * d->prev_q;
            d->prev_i = dec_i; d->prev_q = dec_q;
            float ar = fabsf(del_i), aq = fabsf(del_q);         /* :320-337 */
            if (ar >= aq) {
                if (del_i >= 0.0f) { b0 = '0'; b1 = '0'; } else { b0 = '1'; b1 = '1'; }
            } else {
                if (del_q >= 0.0f) { b0 = '0'; b1 = '1'; } else { b0 = '1'; b1 = '0'; }
            }
        } else {                                                  /* :304-318 */
            if (dec_i < 0.0f) {
                if (dec_q < 0.0f) { b0 = '0'; b1 = '0'; } else { b0 = '0'; b1 = '1'; }
            } else {
                if (dec_q >= 0.0f) { b0 = '1'; b1 = '1'; } else { b0 = '1'; b1 = '0'; }
            }
        }
        if (nb + 2 <= cap) { bits[nb] = b0; bits[nb + 1] = b1; }
        nb += 2;
    }
    if (n_syms_out) *n_syms_out = nsym;
    return nb;
}

/* TSC strip (:413-422): returns index of first char after the TSC, or -1 */
static long tsc_start(const or_demod *d, const char *rx, long n)
{
    if (!d->tsc) return 0;
    long m = d->tsc_len;
    for (long i = 0; i + m <= n; i++)
        if (memcmp(rx + i, d->tsc, (size_t)m) == 0) {
            long s = i + m;
            return s > n ? -1 : s;
        }
    return -1;
}

long or_demod_demodulate_ex(or_demod *d, const float *iq, long n_floats, char *bits, long cap,
                            float *syms, long syms_cap_floats, long *n_syms, long *tsc_idx)
{
    if (n_floats & 1) return -1;                                  /* :347-348 */
    if (n_syms) *n_syms = 0;
    if (tsc_idx) *tsc_idx = 0;
    if (n_floats == 0) return 0;                                  /* :350-351 */
    long nb = demod_core(d, iq, n_floats, bits, cap, syms, syms_cap_floats, n_syms);
    if (nb < 0) return nb;
    if (tsc_idx) *tsc_idx = tsc_start(d, bits, nb < cap ? nb : cap);
    return nb;
}

long or_demod_demodulate(or_demod *d, const float *iq, long n_floats, char *bits, long cap)
{
    if (n_floats & 1) return -1;
    if (n_floats == 0) return 0;
    long need = n_floats + 16;
    if (d->bits_cap < need) {
        d->bits = (char *)realloc(d->bits, (size_t)need);
        d->bits_cap = need;
    }
    long nb = demod_core(d, iq, n_floats, d->bits, d->bits_cap, NULL, 0, NULL);
    if (nb < 0) return nb;
    long s = tsc_start(d, d->bits, nb);
    if (s < 0) return 0;
    long n = nb - s;
    if (n > cap) n = cap;
    memcpy(bits, d->bits + s, (size_t)n);
    return nb - s;
}

long or_demod_constellation(or_demod *d, const float *iq, long n_floats, float *out, long cap)
{
    if (n_floats & 1) return -1;                                  /* :430 */
    ensure_tmp(d, n_floats > 0 ? n_floats : 1);
    const float *src = iq;
    if (d->cfg.iq_balance) {
        or_iqb_process(&d->iqb, src, d->tmp_iqb, n_floats, 0);
        src = d->tmp_iqb;
    }
    if (d->cfg.enable_fll) {
        or_fll_process(d->fll, src, d->tmp_fll, n_floats >> 1);
        src = d->tmp_fll;
    }
    or_cfir_filter(d->rrc, src, d->tmp_rrc, n_floats >> 1);
    long nsym = or_mm_process(d->mm, d->tmp_rrc, n_floats, d->tmp_sym, n_floats);
    if (nsym < 0) return nsym;
    for (long k = 0; k < nsym; k++) {
        float ri, rq;
        or_costas_process(d->costas, d->tmp_sym[2 * k], d->tmp_sym[2 * k + 1], &ri, &rq);
        if (2 * k + 1 < cap) { out[2 * k] = ri; out[2 * k + 1] = rq; }
    }
    return nsym;
}

/* ---- framer (:74-259) ---- */
static void ring_clear(or_demod *d) { d->rb_head = 0; d->rb_count = 0; }

static long ring_tail(const or_demod *d)
{
    long t = d->rb_head - d->rb_count;
    if (t < 0) t += d->ring_cap;
    return t;
}

static uint8_t ring_at(const or_demod *d, long i) { return d->ring[(ring_tail(d) + i) % d->ring_cap]; }

static int ring_write(or_demod *d, uint8_t b)
{
    if (d->rb_count >= d->ring_cap) return 0;
    d->ring[d->rb_head] = b;
    d->rb_head++;
    if (d->rb_head == d->ring_cap) d->rb_head = 0;
    d->rb_count++;
    return 1;
}

static long ring_append_bits(or_demod *d, const char *bits, long n)
{
    long produced = 0;
    for (long i = 0; i < n; i++) {
        d->pack_byte = (uint8_t)((d->pack_byte << 1) | (bits[i] == '1' ? 1 : 0));
        d->pack_bits++;
        if (d->pack_bits == 8) {
            if (!ring_write(d, d->pack_byte)) return -1;
            produced++;
            d->pack_bits = 0;
            d->pack_byte = 0;
        }
    }
    return produced;
}

static long ring_index_of(const or_demod *d, const uint8_t *pat, long np, long from)
{
    if (np == 0) return 0;
    if (d->rb_count < np) return -1;
    long last = d->rb_count - np;
    for (long i = from > 0 ? from : 0; i <= last; i++) {
        int ok = 1;
        for (long j = 0; j < np; j++)
            if (ring_at(d, i + j) != pat[j]) { ok = 0; break; }
        if (ok) return i;
    }
    return -1;
}

static long ring_copy_out(const or_demod *d, long len, uint8_t *out, long cap)
{
    for (long i = 0; i < len && i < cap; i++) out[i] = ring_at(d, i);
    return len;
}

static void reset_framer(or_demod *d)
{
    d->in_frame = 0;
    d->locked_off = -1;
    d->carry_len = 0;
    ring_clear(d);
    d->pack_byte = 0;
    d->pack_bits = 0;
}

long or_demod_bytes(or_demod *d, const float *iq, long n_floats, const uint8_t *start, int n_start,
                    const uint8_t *end, int n_end, uint8_t *out, long cap)
{
    if (n_start == 0 || n_end == 0) return -2;                    /* :174-175 */
    if (n_floats & 1) return -1;
    if (!d->ring) d->ring = (uint8_t *)malloc((size_t)d->ring_cap);
    long need = n_floats + 16;
    char *rx = (char *)malloc((size_t)need);
    long n_rx = or_demod_demodulate(d, iq, n_floats, rx, need);  /* :178 */
    long result = 0;
    if (n_rx <= 0) { free(rx); return n_rx < 0 ? n_rx : 0; }
    if (!d->in_frame) {
        long nc = d->carry_len + n_rx;                            /* :185 */
        char *cand = (char *)malloc((size_t)nc + 1);
        if (d->carry_len) memcpy(cand, d->carry, (size_t)d->carry_len);
        memcpy(cand + d->carry_len, rx, (size_t)n_rx);
        uint8_t *bytes = (uint8_t *)malloc((size_t)(nc / 8 + 1));
        int found = 0;
        for (int off = 0; off < 8 && !found; off++) {            /* :187-230 */
            long nb = or_bits_to_bytes(cand, nc, off, bytes, nc / 8 + 1);
            if (nb <= 0) continue;
            long s = or_index_of(bytes, nb, start, n_start);
            if (s < 0) continue;
            long mend = off + 8 * (s + n_start);
            if (mend > nc) continue;
            found = 1;
            d->in_frame = 1;
            d->locked_off = off;
            ring_clear(d);
            d->pack_byte = 0;
            d->pack_bits = 0;
            long appended = ring_append_bits(d, cand + mend, nc - mend);
            if (appended < 0) { reset_framer(d); result = 0; break; }
            long from = d->rb_count - (appended + n_end);
            long end_at = ring_index_of(d, end, n_end, from > 0 ? from : 0);
            if (end_at >= 0) {
                result = ring_copy_out(d, end_at, out, cap);
                reset_framer(d);
            }
        }
        if (!found) {                                              /* :233-235 */
            long keep = 8L * n_start + 7;
            if (keep > nc) keep = nc;
            char *nc_buf = (char *)malloc((size_t)keep + 1);
            memcpy(nc_buf, cand + nc - keep, (size_t)keep);
            free(d->carry);
            d->carry = nc_buf;
            d->carry_len = keep;
        }
        free(bytes);
        free(cand);
        free(rx);
        return result;
    }
    {                                                              /* :239-258 */
        long appended = ring_append_bits(d, rx, n_rx);
        free(rx);
        if (appended < 0) { reset_framer(d); return 0; }
        long from = d->rb_count - (appended + n_end);
        long end_at = ring_index_of(d, end, n_end, from > 0 ? from : 0);
        if (end_at >= 0) {
            result = ring_copy_out(d, end_at, out, cap);
            reset_framer(d);
        }
        return result;
    }
}

/* ------------------------------------------------------------------------ */
/* Batched CPU baseline (one reference instance per stream, pthreads)         */
/* ------------------------------------------------------------------------ */
typedef struct {
    const or_demod_cfg *cfg;
    const float *iq;
    long stride, n_floats;
    char *bits;
    long bits_cap;
    long *n_bits;
    int s0, s1;
    int rc;
} batch_job;

static void *batch_worker(void *arg)
{
    batch_job *j = (batch_job *)arg;
    for (int s = j->s0; s < j->s1; s++) {
        int err;
        or_demod *d = or_demod_new(j->cfg, &err);
        if (!d) { j->rc = err; return NULL; }
        char *tmp = (char *)malloc((size_t)j->n_floats + 16);
        long nb = demod_core(d, j->iq + (long)s * j->stride, j->n_floats, tmp, j->n_floats + 16,
                             NULL, 0, NULL);
        long st = tsc_start(d, tmp, nb);
        long n = st < 0 ? 0 : nb - st;
        if (j->n_bits) j->n_bits[s] = n;
        if (j->bits && n > 0) memcpy(j->bits + (long)s * j->bits_cap, tmp + st,
                                     (size_t)(n < j->bits_cap ? n : j->bits_cap));
        free(tmp);
        or_demod_free(d);
    }
    return NULL;
}

/* Packed variant for the bench's parity-at-scale check and the all-core CPU
 * baseline: the raw (pre-TSC) bits of one DeModulate call per stream, packed
 * MSB-first exactly like the GPU bit rows (BitPacker order, HelperFunctions.cs:14-29),
 * plus optionally the rotated Costas symbols.  Streams are handed out through
 * an atomic counter (any thread count, no static partition).  bits / syms may
 * be NULL (timing only). */
typedef struct {
    const or_demod_cfg *cfg;
    const float *iq;
    long stride, n_floats;
    uint8_t *bits;
    long bits_stride;
    long *n_bits;
    float *syms;
    long syms_stride;
    long *n_syms;
    int n_streams;
    int *next;
    int rc;
} packed_job;

static void *packed_worker(void *arg)
{
    packed_job *j = (packed_job *)arg;
    char *tmp = (char *)malloc((size_t)j->n_floats + 16);
    for (;;) {
        int s = __atomic_fetch_add(j->next, 1, __ATOMIC_RELAXED);
        if (s >= j->n_streams) break;
        int err;
        or_demod *d = or_demod_new(j->cfg, &err);
        if (!d) { j->rc = err ? err : -1; break; }
        long ns = 0;
        float *srow = j->syms ? j->syms + (long)s * j->syms_stride : NULL;
        long nb = 0;
        if (j->n_floats > 0)
            nb = demod_core(d, j->iq + (long)s * j->stride, j->n_floats, tmp, j->n_floats + 16, srow,
                            j->syms ? j->syms_stride : 0, &ns);
        if (j->n_bits) j->n_bits[s] = nb;
        if (j->n_syms) j->n_syms[s] = ns;
        if (j->bits) {
            uint8_t *row = j->bits + (long)s * j->bits_stride;
            long nbytes = (nb + 7) / 8;
            if (nbytes > j->bits_stride) nbytes = j->bits_stride;
            memset(row, 0, (size_t)nbytes);
            for (long i = 0; i < nb && (i >> 3) < nbytes; i++)
                if (tmp[i] == '1') row[i >> 3] |= (uint8_t)(0x80u >> (i & 7));
        }
        or_demod_free(d);
    }
    free(tmp);
    return NULL;
}

int or_demod_batch_packed(const or_demod_cfg *cfg, int n_streams, const float *iq, long stride_floats,
                          long n_floats, uint8_t *bits, long bits_stride, long *n_bits, float *syms,
                          long syms_stride_floats, long *n_syms, int n_threads)
{
    if (n_floats & 1) return -1;
    if (n_threads < 1) n_threads = 1;
    if (n_threads > n_streams) n_threads = n_streams > 0 ? n_streams : 1;
    pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
    packed_job *jobs = (packed_job *)calloc((size_t)n_threads, sizeof(packed_job));
    int next = 0;
    for (int t = 0; t < n_threads; t++) {
        packed_job *j = &jobs[t];
        j->cfg = cfg; j->iq = iq; j->stride = stride_floats; j->n_floats = n_floats;
        j->bits = bits; j->bits_stride = bits_stride; j->n_bits = n_bits;
        j->syms = syms; j->syms_stride = syms_stride_floats; j->n_syms = n_syms;
        j->n_streams = n_streams; j->next = &next; j->rc = 0;
        pthread_create(&th[t], NULL, packed_worker, j);
    }
    int rc = 0;
    for (int t = 0; t < n_threads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].rc) rc = jobs[t].rc;
    }
    free(th);
    free(jobs);
    return rc;
}

int or_demod_batch(const or_demod_cfg *cfg, int n_streams, const float *iq, long stride_floats,
                   long n_floats, char *bits_out, long bits_cap, long *n_bits, int n_threads)
{
    if (n_threads < 1) n_threads = 1;
    if (n_threads > n_streams) n_threads = n_streams > 0 ? n_streams : 1;
    pthread_t th[256];
    batch_job jobs[256];
    if (n_threads > 256) n_threads = 256;
    for (int t = 0; t < n_threads; t++) {
        batch_job *j = &jobs[t];
        j->cfg = cfg; j->iq = iq; j->stride = stride_floats; j->n_floats = n_floats;
        j->bits = bits_out; j->bits_cap = bits_cap; j->n_bits = n_bits;
        j->s0 = (int)((long)n_streams * t / n_threads);
        j->s1 = (int)((long)n_streams * (t + 1) / n_threads);
        j->rc = 0;
        pthread_create(&th[t], NULL, batch_worker, j);
    }
    int rc = 0;
    for (int t = 0; t < n_threads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].rc) rc = jobs[t].rc;
    }
    return rc;
}

/* ------------------------------------------------------------------------ */
/* Input synthesis                                                           */
/* ------------------------------------------------------------------------ */
uint64_t or_splitmix64(uint64_t *state)
{
    uint64_t z = (*state += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static double next_double(uint64_t *st) { return (double)(or_splitmix64(st) >> 11) * 0x1.0p-53; }

/* QPSKModulator.cs:104-167 */
long or_modulate(int sample_rate, int symbol_rate, double rrc_alpha, int rrc_span, int differential,
                 const char *tsc, const char *bits, long n_bits, int pulse_shaping, float *out,
                 long cap_floats)
{
    double taps[4096];
    int nt = or_rrc_taps((double)rrc_span, rrc_alpha, sample_rate, symbol_rate, taps, 4096);
    if (nt <= 0) return -1;
    float tf[4096];
    for (int i = 0; i < nt; i++) tf[i] = (float)taps[i];       /* ToInterleavedIQRealTapsStatic */
    long tl = is_blank(tsc) ? 0 : (long)strlen(tsc);
    long total_bits = tl + n_bits;
    long nd = total_bits >> 1;
    if (nd == 0) return 0;
    int sps = sample_rate / symbol_rate;
    if (sps <= 0) return -1;
    long delay = (nt - 1) / 2;
    long base_c = delay + nd * sps;
    long total = pulse_shaping ? base_c + delay : base_c;
    if (2 * total > cap_floats) return -(2 * total);
    const float inv_sqrt2 = 0.7071067811865475f;
    float *up = (float *)calloc((size_t)(2 * total), sizeof(float));
    float pi_ = inv_sqrt2, pq = inv_sqrt2;
    long w = delay;
    for (long dd = 0; dd < nd; dd++) {
        long i0 = 2 * dd, i1 = 2 * dd + 1;
        char c0 = i0 < tl ? tsc[i0] : bits[i0 - tl];
        char c1 = i1 < tl ? tsc[i1] : bits[i1 - tl];
        int bi = c0 - '0', bq = c1 - '0';
        float si, sq;
        if (differential) {
            float di, dq;                                          /* :92-102 */
            if (bi == 0 && bq == 0) { di = 1.0f; dq = 0.0f; }
            else if (bi == 0 && bq == 1) { di = 0.0f; dq = 1.0f; }
            else if (bi == 1 && bq == 1) { di = -1.0f; dq = 0.0f; }
            else { di = 0.0f; dq = -1.0f; }
            si = pi_ * di - pq * dq;
            sq = pi_ * dq + pq * di;
            pi_ = si; pq = sq;
        } else {
            si = bi == 0 ? -inv_sqrt2 : inv_sqrt2;
            sq = bq == 0 ? -inv_sqrt2 : inv_sqrt2;
        }
        up[2 * w] = si;
        up[2 * w + 1] = sq;
        w += sps;
    }
    if (!pulse_shaping) {
        memcpy(out, up, (size_t)(2 * total) * sizeof(float));
        free(up);
        return 2 * total;
    }
    /* fftFilter (FIRFilter.cs:96-141): y[i] = conv(up, h)[T-1+i], double accumulate */
    for (long i = 0; i < total; i++) {
        double ar = 0.0, ai = 0.0;
        long m0 = (nt - 1 + i) - (total - 1);
        if (m0 < 0) m0 = 0;
        for (long m = m0; m < nt; m++) {
            long src = nt - 1 + i - m;
            if (src < 0) break;
            float xr = up[2 * src], xi = up[2 * src + 1];
            if (xr == 0.0f && xi == 0.0f) continue;
            ar += (double)tf[m] * xr;
            ai += (double)tf[m] * xi;
        }
        out[2 * i] = (float)ar;
        out[2 * i + 1] = (float)ai;
    }
    free(up);
    return 2 * total;
}

/* LocalOscilator.cs:5-194 */
struct or_nco {
    double base_hz, fs, max_ppm, static_ppm, drift_ppm, total_ppm, cur_hz, phase;
    int interval, counter;
    uint64_t rng;
};

static void nco_update_freq(or_nco *n) { n->cur_hz = n->base_hz * (1.0 + n->total_ppm * 1e-6); }

static void nco_wrap(or_nco *n)
{
    const double two_pi = 2.0 * OR_PI;
    n->phase = fmod(n->phase, two_pi);
    if (n->phase < 0) n->phase += two_pi;
}

or_nco *or_nco_new(double freq_hz, double fs, double ppm, double phase0, uint64_t seed)
{
    if (fs <= 0) return NULL;
    or_nco *n = (or_nco *)calloc(1, sizeof(*n));
    n->base_hz = freq_hz;
    n->fs = fs;
    n->phase = phase0;
    n->max_ppm = fabs(ppm);
    n->rng = seed;
    double iv = fs * 1e-3;
    n->interval = (int)(iv > 1 ? iv : 1);
    n->counter = 0;
    n->static_ppm = n->max_ppm > 0.0 ? (next_double(&n->rng) * 2.0 - 1.0) * n->max_ppm : 0.0;
    n->drift_ppm = 0.0;
    n->total_ppm = n->static_ppm;
    nco_update_freq(n);
    nco_wrap(n);
    return n;
}

void or_nco_free(or_nco *n) { free(n); }

void or_nco_next(or_nco *n, double *re, double *im)
{
    if (n->max_ppm <= 0.0) {
        n->cur_hz = n->base_hz;
    } else {
        n->counter++;
        if (n->counter >= n->interval) {
            n->counter = 0;
            double step_std = n->max_ppm * 0.001;
            double step = (next_double(&n->rng) * 2.0 - 1.0) * step_std;
            n->drift_ppm += step;
            n->total_ppm = n->static_ppm + n->drift_ppm;
            if (n->total_ppm > n->max_ppm) {
                n->total_ppm = n->max_ppm;
                n->drift_ppm = n->total_ppm - n->static_ppm;
            } else if (n->total_ppm < -n->max_ppm) {
                n->total_ppm = -n->max_ppm;
                n->drift_ppm = n->total_ppm - n->static_ppm;
            }
            nco_update_freq(n);
        }
    }
    double inc = 2.0 * OR_PI * n->cur_hz / n->fs;
    n->phase += inc;
    nco_wrap(n);
    *re = or_libm_cos(n->phase);
    *im = or_libm_sin(n->phase);
}

void or_apply_lo_pair(or_nco *tx, or_nco *rx, float *iq, long n_complex)
{
    for (long i = 0; i < n_complex; i++) {
        double ar, ai, br, bi;
        or_nco_next(tx, &ar, &ai);
        or_nco_next(rx, &br, &bi);
        bi = -bi;                                                  /* Conjugate */
        double lr = (ar * br) - (ai * bi);                         /* System.Numerics.Complex * */
        double li = (ai * br) + (ar * bi);
        double xr = iq[2 * i], xi = iq[2 * i + 1];
        double yr = (xr * lr) - (xi * li);
        double yi = (xi * lr) + (xr * li);
        iq[2 * i] = (float)yr;
        iq[2 * i + 1] = (float)yi;
    }
}

/* Portable sincos (or_sincos.h) over an array, for the test sweeps. */
void or_sincos_batch(const double *x, long n, double *s, double *c)
{
    for (long i = 0; i < n; i++) or_sincos(x[i], &s[i], &c[i]);
}
