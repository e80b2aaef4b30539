// qpsk_design.cpp -- constructor math of QPSKDeModulator (host, once per handle).
// Build with -ffp-contract=off: the C# never fuses a*b+c.
#include "qpsk_design.h"

#include <cmath>

#include "qpsk_demod.h"

namespace qpsk {

namespace {
constexpr double kPi = 3.14159265358979311600;     // Math.PI
constexpr float kPiF = 3.14159274101257324219f;    // MathF.PI
// Math.Pow is a libm call in .NET; keep the compiler from folding pow(x, 2.0)
// into x*x (libm pow(x, 2.0) is not always the correctly rounded x*x).
double (*volatile libm_pow)(double, double) = std::pow;

// Band-Edge Filter.cs:197-202
float band_edge_sinc(float x) {
    if (x == 0.0f) return 1.0f;
    float arg = kPiF * x;
    return std::sin(arg) / arg;
}
}  // namespace

std::vector<double> rrc_coefficients(double span_symbols, double beta, int sample_rate,
                                     int symbol_rate) {
    const double sps_exact = static_cast<double>(sample_rate) / symbol_rate;  // RRC-filter.cs:24
    const int sps = static_cast<int>(std::nearbyint(sps_exact));              // Math.Round (half-even)
    const int span = static_cast<int>(std::nearbyint(span_symbols));          // :26
    const int taps = span * sps + 1;                                          // :27
    if (taps <= 0) return {};
    std::vector<double> h(taps);
    const int mid = (taps - 1) / 2;
    const double eps = 1e-8;
    for (int n = 0; n < taps; ++n) {
        const double t = (n - mid) / static_cast<double>(sps);               // :38
        double v;
        if (std::fabs(t) < eps) {                                            // t = 0
            v = 1.0 + beta * (4.0 / kPi - 1.0);
        } else if (std::fabs(std::fabs(t) - 1.0 / (4.0 * beta)) < eps) {     // t = +-1/(4 beta)
            v = (beta / std::sqrt(2.0)) * ((1.0 + 2.0 / kPi) * std::sin(kPi / (4.0 * beta)) +
                                           (1.0 - 2.0 / kPi) * std::cos(kPi / (4.0 * beta)));
        } else {
            const double num =
                std::sin(kPi * t * (1.0 - beta)) + 4.0 * beta * t * std::cos(kPi * t * (1.0 + beta));
            const double den = kPi * t * (1.0 - libm_pow(4.0 * beta * t, 2.0));
            v = num / den;
        }
        h[n] = v;
    }
    double energy = 0.0;                                                     // :65-72
    for (double v : h) energy += v * v;
    const double norm = std::sqrt(energy);
    for (double &v : h) v /= norm;
    return h;
}

int design_loops(int sample_rate, int symbol_rate, float rrc_alpha, int rrc_span,
                 double symbol_sync_bw, double costas_loop_bw, double cfo_loop_bw,
                 LoopDesign *out, std::string *err) {
    if (symbol_rate <= 0) {
        *err = "SymbolRate must be positive (the reference divides by it)";
        return QPSK_ERR_ARGUMENT;
    }
    // QPSKDeModulator.cs:28-32: RRC taps from the float alpha widened to double.
    std::vector<double> h = rrc_coefficients(static_cast<double>(rrc_span),
                                             static_cast<double>(rrc_alpha), sample_rate,
                                             symbol_rate);
    if (h.empty() || h.size() > 4096) {
        *err = "rrcSpan * samples-per-symbol gives an unsupported tap count";
        return QPSK_ERR_ARGUMENT;
    }
    out->rrc_f32.resize(h.size());
    for (size_t i = 0; i < h.size(); ++i) out->rrc_f32[i] = static_cast<float>(h[i]);  // :284

    // QPSKDeModulator.cs:35: FLLBandEdgeFilter(SampleRate / SymbolRate, RrcAlpha, 40,
    // (float)CFOLoopBandwith), validated in its ctor (Band-Edge Filter.cs:42-45).
    const float fsps = static_cast<float>(sample_rate / symbol_rate);
    const float rolloff = rrc_alpha;
    const int ntaps = 40;
    const float bw = static_cast<float>(cfo_loop_bw);
    if (fsps <= 0.0f) { *err = "sps must be > 0."; return QPSK_ERR_OUT_OF_RANGE; }
    if (rolloff < 0 || rolloff > 1.0f) { *err = "rolloff must be in [0,1]."; return QPSK_ERR_OUT_OF_RANGE; }
    if (bw <= 0.0f) { *err = "bandwidth must be > 0."; return QPSK_ERR_OUT_OF_RANGE; }
    const float two_pi_f = 2.0f * kPiF;
    out->fll_sps = fsps;
    out->fll_alpha = 0.0f;
    out->fll_beta = 4.0f * bw / fsps;                                        // :56
    out->fll_max_freq = two_pi_f * (2.0f / fsps);                            // :58
    out->fll_taps = ntaps;
    {   // DesignFilter, Band-Edge Filter.cs:132-183
        const int mid = (ntaps - 1) / 2;
        std::vector<float> bb(ntaps);
        float sum = 0.0f;
        for (int i = 0; i < ntaps; ++i) {
            const float k = static_cast<float>(i - mid) / (2.0f * fsps);
            const float pos = rolloff * k;
            const float tap = band_edge_sinc(pos - 0.5f) + band_edge_sinc(pos + 0.5f);
            sum += tap;
            bb[i] = tap;
        }
        for (int i = 0; i < ntaps; ++i) bb[i] /= sum;
        out->fll_lower_iq.assign(2 * ntaps, 0.0f);
        out->fll_upper_iq.assign(2 * ntaps, 0.0f);
        for (int i = 0; i < ntaps; ++i) {
            const float k = static_cast<float>(i - mid) / (2.0f * fsps);
            const float angle = -two_pi_f * (1.0f + rolloff) * k;
            const float wc = std::cos(angle);
            const float ws = std::sin(angle);
            const float li = bb[i] * wc;
            const float lq = bb[i] * ws;
            out->fll_lower_iq[2 * i] = li;
            out->fll_lower_iq[2 * i + 1] = lq;
            out->fll_upper_iq[2 * i] = li;       // upper = conj(lower)
            out->fll_upper_iq[2 * i + 1] = -lq;
        }
    }
    {   // setupSymbolSync, QPSKDeModulator.cs:39-55
        const double zeta = 1.0 / std::sqrt(2.0);
        const double bn = symbol_sync_bw;
        const double wn = ((2.0 * kPi * bn) / (zeta + 0.25) / zeta);
        const double denom = 1.0 + 2.0 * zeta * wn + wn * wn;
        out->kp = (4.0 * zeta * wn) / denom;
        out->ki = (4.0 * wn * wn) / denom;
        out->mm_sps = static_cast<double>(sample_rate) / static_cast<double>(symbol_rate);
    }
    {   // CostasLoopQpsk(SymbolRate, SymbolRate / CostasLoopBandwith), CostasLoopQpsk.cs:29-48
        const double fs = static_cast<double>(symbol_rate);
        const double loop_bw_hz = static_cast<double>(symbol_rate) / costas_loop_bw;
        const double damping = 0.707;
        const double bwn = 2.0 * kPi * loop_bw_hz / fs;
        const double d = 1.0 + 2.0 * damping * bwn + bwn * bwn;
        out->costas_alpha = (4.0 * damping * bwn) / d;
        out->costas_beta = (4.0 * bwn * bwn) / d;
    }
    return QPSK_OK;
}

}  // namespace qpsk
