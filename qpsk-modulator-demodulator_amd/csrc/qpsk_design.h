// qpsk_design.h -- host-side constructor math of the reference QPSKDeModulator:
// RRC taps, Mueller-Muller / Costas loop gains, Band-Edge FLL taps and gains.
// Runs once per handle; compiled with -ffp-contract=off so every double/float
// operation rounds exactly as the C# does.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace qpsk {

// RRC-filter.cs:16-75 (generateCoefficents); double precision, unit energy.
std::vector<double> rrc_coefficients(double span_symbols, double beta, int sample_rate,
                                     int symbol_rate);

struct LoopDesign {
    // MuellerMuller (QPSKDeModulator.cs:39-55)
    double mm_sps = 0, kp = 0, ki = 0;
    // CostasLoopQpsk (QPSKDeModulator.cs:56, CostasLoopQpsk.cs:29-48)
    double costas_alpha = 0, costas_beta = 0;
    // FLLBandEdgeFilter (QPSKDeModulator.cs:35, Band-Edge Filter.cs:40-62)
    float fll_sps = 0, fll_beta = 0, fll_alpha = 0, fll_max_freq = 0;
    int fll_taps = 40;
    std::vector<float> fll_lower_iq, fll_upper_iq;  // interleaved complex taps
    std::vector<float> rrc_f32;                      // (float) RRC taps, imag = 0
};

// Returns 0 or a QPSK_ERR_* code; message in *err.
int design_loops(int sample_rate, int symbol_rate, float rrc_alpha, int rrc_span,
                 double symbol_sync_bw, double costas_loop_bw, double cfo_loop_bw,
                 LoopDesign *out, std::string *err);

}  // namespace qpsk
