/*
 * qpsk_oracle.h -- CPU restatement of the reference C# demodulation chain.
 *
 * TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg, never by the product library.
 *
 * Parity status: the reference is C# (.NET 9) and no .NET runtime exists in
 * this image or on the GPU box, so the oracle cannot be compared with the C#
 * itself, and the reference ships no golden vectors.  Bit-level parity with the
 * C# is therefore UNPINNED; the restatement is cross-checked by an
 * independent numpy/Python model (tests/refmodel.py) and by the reference's
 * only known-answer check, testAtDataLevel.cs:46 (payload recovery).
 *
 * Every function cites the reference file:line it restates.
 */
#ifndef QPSK_ORACLE_H
#define QPSK_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* trig_mode: 0 = libm (glibc cos/sin/cosf/sinf, what .NET-on-Linux calls),
 *            1 = portable (or_sincos.h, bit-identical to the GPU path)      */
#define OR_TRIG_LIBM 0
#define OR_TRIG_PORTABLE 1

/* RRC-filter.cs:16-75 */
int or_rrc_taps(double span_symbols, double beta, int sample_rate, int symbol_rate,
                double *out, int cap);

/* FIRFilter.cs:8-232 (ComplexFIRFilter; lanes = Vector<float>.Count, 0/1 = scalar path) */
typedef struct or_cfir or_cfir;
or_cfir *or_cfir_new(const float *taps_iq, int n_floats, int lanes);
void or_cfir_free(or_cfir *f);
void or_cfir_filter(or_cfir *f, const float *in_iq, float *out_iq, long n_complex);

/* MuellerMuller.cs:17-249 */
typedef struct or_mm or_mm;
/* the C# path would throw IndexOutOfRangeException (see or_mm_process) */
#define OR_ERR_INDEX (-3)
or_mm *or_mm_new(double sps, double kp, double ki);
void or_mm_free(or_mm *m);
long or_mm_process(or_mm *m, const float *in_iq, long n_floats, float *out_iq, long out_floats);

/* CostasLoopQpsk.cs:19-130 */
typedef struct or_costas or_costas;
or_costas *or_costas_new(double sample_rate, double loop_bw_hz, double damping, int trig_mode);
void or_costas_free(or_costas *c);
void or_costas_process(or_costas *c, float in_i, float in_q, float *out_i, float *out_q);
void or_costas_state(const or_costas *c, double *theta, double *freq);

/* Band-Edge Filter.cs:14-203 */
typedef struct or_fll or_fll;
or_fll *or_fll_new(float sps, float rolloff, int filter_size, float bandwidth, int lanes,
                   int trig_mode);
void or_fll_free(or_fll *f);
void or_fll_process(or_fll *f, const float *in_iq, float *out_iq, long n_complex);
int or_fll_taps(const or_fll *f, float *lower_iq, float *upper_iq, int cap_floats);
void or_fll_state(const or_fll *f, float *phase, float *freq);

/* QPSKDeModulator.cs:11-457 */
/* IQ_Balancer (IQ Balancer.cs:10-26): a DC blocker, exponential averages of I
 * and Q with ratio 1e-5f.  literal = 1 keeps the reference loop bound
 * (i < IN.Length/2 floats: the first half of the complex samples; the rest of
 * OUT is not written), 0 covers the whole buffer. */
typedef struct { float avg_re, avg_im; } or_iqb;
void or_iqb_process(or_iqb *b, const float *in_iq, float *out_iq, long n_floats, int literal);
typedef struct or_demod or_demod;
typedef struct or_demod_cfg {
    int sample_rate, symbol_rate;
    float rrc_alpha;
    int rrc_span;
    double symbol_sync_bw, costas_loop_bw, cfo_loop_bw;
    int differential;
    const char *tsc;       /* NULL / whitespace-only = no TSC (QPSKDeModulator.cs:21) */
    int enable_fll;        /* 0 = reference DeModulate (fll.Process commented out, :359) */
    int lanes;             /* Vector<float>.Count (8 on AVX2 x64) */
    int trig_mode;
    long ring_capacity;    /* framer ring bytes; reference uses 300_000_000 (:58) */
    int iq_balance;        /* 0 = off (the reference constructs IQ_Balancer, :38, but never
                              calls it); 1 = IQ_Balancer.Process over the whole call before
                              the FLL / matched filter (loop bound fixed) */
} or_demod_cfg;
void or_demod_cfg_default(or_demod_cfg *c, int sample_rate, int symbol_rate);
/* returns NULL and sets *err (1 = ArgumentOutOfRange from FLL validation) on error */
or_demod *or_demod_new(const or_demod_cfg *cfg, int *err);
void or_demod_free(or_demod *d);
/* DeModulate (:345-425): writes '0'/'1' chars, returns count; -1 odd length */
long or_demod_demodulate(or_demod *d, const float *iq, long n_floats, char *bits, long cap);
/* raw bits before TSC strip and the symbol (constellation) output of the same call */
long or_demod_demodulate_ex(or_demod *d, const float *iq, long n_floats, char *bits, long cap,
                            float *syms, long syms_cap_floats, long *n_syms, long *tsc_idx);
/* deModulateConstellation (:427-455) */
long or_demod_constellation(or_demod *d, const float *iq, long n_floats, float *out, long cap);
/* DeModulateBytes (:169-259): returns payload length (0 = none), -1 odd, -2 empty marker */
long or_demod_bytes(or_demod *d, const float *iq, long n_floats, const uint8_t *start, int n_start,
                    const uint8_t *end, int n_end, uint8_t *out, long cap);
/* design products, for cross-checks */
void or_demod_gains(const or_demod *d, double *mm_sps, double *kp, double *ki, double *c_alpha,
                    double *c_beta);
int or_demod_rrc_f32(const or_demod *d, float *taps, int cap);

/* Framer pieces on a bit string (HelperFunctions.cs:11-71) */
long or_bits_to_bytes(const char *bits, long n_bits, int bit_offset, uint8_t *out, long cap);
long or_index_of(const uint8_t *hay, long n_hay, const uint8_t *needle, long n_needle);

/* Batched baseline: S independent reference demodulators, one per stream,
 * spread over n_threads pthreads.  iq is [S][stride_floats]; each stream gets
 * one DeModulate call of n_floats.  bits_out is [S][bits_cap] chars. */
int or_demod_batch(const or_demod_cfg *cfg, int n_streams, const float *iq, long stride_floats,
                   long n_floats, char *bits_out, long bits_cap, long *n_bits, int n_threads);
/* one DeModulate call per stream, raw bits packed MSB-first into rows of
 * bits_stride bytes (+ optional rotated symbols); work-stealing threads */
int or_demod_batch_packed(const or_demod_cfg *cfg, int n_streams, const float *iq, long stride_floats,
                          long n_floats, uint8_t *bits, long bits_stride, long *n_bits, float *syms,
                          long syms_stride_floats, long *n_syms, int n_threads);

/* Input synthesis (not accelerated): QPSKModulator.cs:104-167 with the MathNet
 * FFT of FIRFilter.cs:96-141 restated as direct double convolution.
 * Parity at this boundary is unpinned (MathNet.Numerics 5.0.0 absent). */
long or_modulate(int sample_rate, int symbol_rate, double rrc_alpha, int rrc_span, int differential,
                 const char *tsc, const char *bits, long n_bits, int pulse_shaping, float *out,
                 long cap_floats);
/* LocalOscilator.cs:5-194 with System.Random replaced by seeded splitmix64 */
typedef struct or_nco or_nco;
or_nco *or_nco_new(double freq_hz, double fs, double ppm, double phase0, uint64_t seed);
void or_nco_free(or_nco *n);
void or_nco_next(or_nco *n, double *re, double *im);
/* testAtDataLevel.cs:39-42: iq[i] *= tx.Next() * conj(rx.Next()) in double, cast to float */
void or_apply_lo_pair(or_nco *tx, or_nco *rx, float *iq, long n_complex);
uint64_t or_splitmix64(uint64_t *state);
void or_sincos_batch(const double *x, long n, double *s, double *c);

#ifdef __cplusplus
}
#endif
#endif
