// qpsk_state.h -- per-stream loop state kept in HBM between process() calls,
// and the uniform launch parameters of the loop kernels.
//
// One StreamState per stream = the private fields of one reference
// QPSKDeModulator instance:
//   MuellerMuller.cs:24-36      baseIndex, mu, ncoIntegral, prev sample/decision
//   CostasLoopQpsk.cs:25-27     theta, freq
//   QPSKDeModulator.cs:72-73    differential-decoder previous decision
//   Band-Edge Filter.cs:25-26   FLL phase, freq (+ the 40-sample delay line, kept
//                               in its own array)
// The M&M sample queue (MuellerMuller.cs:32-36) is kept as the count of
// retained matched-filter samples plus those samples in a carry array.
#pragma once
#include <cstdint>

namespace qpsk {

// retained M&M samples between calls: at most 3 whatever sps is
// (MuellerMuller.cs:123-133 drops min(baseIndex - 1, count - 3), and the loop
// leaves baseIndex >= count - 2); more only when the output capacity stops the
// loop early (sps below ~1, where DeModulate's n-symbol span is too small)
constexpr int kCarryMax = 256;
constexpr int kMfPrefix = 256;     // MF buffer prefix that receives the carry
constexpr int kFllTaps = 40;       // QPSKDeModulator.cs:35

struct alignas(16) StreamState {
    double mu;          // MuellerMuller.mu
    double integ;       // MuellerMuller.ncoIntegral
    double theta;       // CostasLoopQpsk.theta
    double freq;        // CostasLoopQpsk.freq
    int32_t base;       // MuellerMuller.baseIndex (relative to the retained queue)
    int32_t has_prev;   // MuellerMuller.hasPrev
    float psi, psq;     // MuellerMuller.prevSample
    float pdi, pdq;     // MuellerMuller.prevDecision
    int32_t carry_n;    // retained queue length (_bufCount after the last call)
    int32_t diff_have;  // QPSKDeModulator._diffHavePrev
    float diff_pi, diff_pq;
    float fll_phase, fll_freq;
    int32_t fll_pos;    // FLL delay-line write position
    int32_t error;      // sticky: 1 = carry overflow
    int64_t tofs;       // inside a call split into internal chunks: index of this
                        // chunk's queue start in the whole call's M&M queue, so
                        // the timing arithmetic runs at the reference's absolute
                        // baseIndex (0 between calls)
    float iqb_re, iqb_im;   // IQ_Balancer._avgReal, _avgImg (IQ Balancer.cs:13)
};

struct LoopParams {
    double sps, kp, ki;            // MuellerMuller
    double c_alpha, c_beta;        // CostasLoopQpsk
    int32_t differential;
    int32_t costas_trig;           // 0 portable table sincos, 1 glibc sin/cos (qpsk_glibc_trig.h)
};

struct FllParams {
    float beta, alpha, max_freq, min_freq;
    float lower_rev[2 * kFllTaps]; // interleaved complex taps, reversed
    float upper_rev[2 * kFllTaps]; // (ComplexFIRFilter ctor, FIRFilter.cs:43-48)
    int32_t lanes;
    int32_t conj_taps;             // upper_rev == conj(lower_rev) bit for bit (the reference design)
};

}  // namespace qpsk
