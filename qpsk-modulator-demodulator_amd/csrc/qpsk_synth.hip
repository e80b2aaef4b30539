// qpsk_synth.hip -- batched synthetic baseband on the GPU (the reference's
// QPSKModulator.Modulate, QPSKModulator.cs:104-167, plus the test-bench channel
// of testAtDataLevel.cs:27-42 / testFullDemodChain.cs:64-75), so multi-GiB
// inputs never cross PCIe.
//
//   synth_symbols_kernel  one lane per stream: payload dibits from
//                         splitmix64(seed ^ stream), differential mapping
//                         (DibitToDelta, :92-102; reference point (1/sqrt2)(1+j))
//                         kept as a quadrant index 0..3.
//   synth_samples_kernel  one thread per output sample: RRC pulse shaping
//                         (the FFT filter of FIRFilter.cs:96-141 as a direct
//                         polyphase sum in double, symbol d peaking at d*sps),
//                         optional 4-tap multipath folded into the pulse, carrier
//                         offset e^{j(2 pi f n / fs + phi0)}, AWGN (Box-Muller,
//                         HelperModels.cs:27-34) from a counter-based hash.
// Not on the parity path: the demodulator and the oracle consume the same
// generated buffer.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "qpsk_demod.h"
#include "qpsk_design.h"

namespace {

__host__ __device__ inline uint64_t splitmix64(uint64_t &st) {
    uint64_t z = (st += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__host__ __device__ inline double u01(uint64_t v) { return static_cast<double>(v >> 11) * 0x1.0p-53; }

struct SynthArgs {
    int S;
    int64_t n;            // samples per stream
    int64_t nsym;         // symbols per stream
    int sps;
    int mid;              // (T-1)/2
    int G;                // composite pulse length (T + multipath taps - 1)
    uint64_t seed;
    int64_t s0;           // global id of row 0 (qpsk_synth_params.first_stream)
    double cfo_hz, lo_ppm, lo_hz, fs;
    double noise_sigma;   // per component, 0 = none
    int differential;
    int carrier;          // 0: lo_ppm = cfo_hz = 0, the modulator's own baseband
    uint8_t *quad;        // [S][nsym] quadrant / symbol index
    uint8_t *bits;        // [S][bits_stride] payload bits MSB-first
    int64_t bits_stride;
    float *iq;            // [S][stride] float2
    int64_t stride;       // floats
};

struct Pulse {
    double re[300];
    double im[300];
};

__global__ void synth_symbols_kernel(SynthArgs a) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= a.S) return;
    const uint64_t gs = static_cast<uint64_t>(a.s0 + s);
    uint64_t rng = a.seed ^ (0x5159534BULL + gs * 0x9E3779B97F4A7C15ULL);
    uint8_t *q = a.quad + s * a.nsym;
    uint8_t *b = a.bits ? a.bits + s * a.bits_stride : nullptr;
    // quadrant k <-> (cos, sin)(pi/4 + k pi/2); reference (1/sqrt2)(1+j) = 0
    int quad = 0;
    uint64_t word = 0;
    int left = 0;
    for (int64_t d = 0; d < a.nsym; ++d) {
        if (left == 0) { word = splitmix64(rng); left = 32; }
        const int dibit = static_cast<int>(word >> 62);
        word <<= 2;
        --left;
        if (b) {
            const int64_t bit = 2 * d;
            uint8_t &byte = b[bit >> 3];
            const int sh = 6 - static_cast<int>(bit & 7);
            byte = static_cast<uint8_t>((byte & ~(3 << sh)) | (dibit << sh));
        }
        if (a.differential) {
            // DibitToDelta: 00 -> +1, 01 -> +j, 11 -> -1, 10 -> -j (rotation by k*90deg)
            const int rot = dibit == 0 ? 0 : dibit == 1 ? 1 : dibit == 3 ? 2 : 3;
            quad = (quad + rot) & 3;
            q[d] = static_cast<uint8_t>(quad);
        } else {
            // bi -> I sign, bq -> Q sign: (+,+)=0, (-,+)=1, (-,-)=2, (+,-)=3
            const int bi = dibit >> 1, bq = dibit & 1;
            q[d] = static_cast<uint8_t>(bi ? (bq ? 0 : 3) : (bq ? 1 : 2));
        }
    }
}

__global__ void synth_samples_kernel(SynthArgs a, Pulse p) {
    const int s = blockIdx.y;
    const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const double c = 0.70710678118654752440;
    const double qre[4] = {c, -c, -c, c};
    const double qim[4] = {c, c, -c, -c};
    const uint8_t *q = a.quad + s * a.nsym;
    // y[i] = sum_d sym_d g[mid + i - d*sps]
    double yr = 0.0, yi = 0.0;
    const int64_t dlo = (i + a.mid - (a.G - 1) + a.sps - 1) / a.sps;
    const int64_t dhi = (i + a.mid) / a.sps;
    for (int64_t d = dlo < 0 ? 0 : dlo; d <= dhi && d < a.nsym; ++d) {
        const int k = static_cast<int>(a.mid + i - d * a.sps);
        if (k < 0 || k >= a.G) continue;
        const int qq = q[d];
        yr += p.re[k] * qre[qq] - p.im[k] * qim[qq];
        yi += p.re[k] * qim[qq] + p.im[k] * qre[qq];
    }
    // per-stream carrier: +-ppm LO pair (testAtDataLevel.cs:27-28) or +-cfo_hz
    const uint64_t gs = static_cast<uint64_t>(a.s0 + s);
    uint64_t rs = a.seed ^ (0xC0FFEE123ULL + gs * 0xD1B54A32D192ED03ULL);
    const double u1 = u01(splitmix64(rs)), u2 = u01(splitmix64(rs)), u3 = u01(splitmix64(rs));
    double f = 0.0;
    if (a.cfo_hz > 0.0) f = (2.0 * u1 - 1.0) * a.cfo_hz;
    else if (a.lo_ppm > 0.0) f = a.lo_hz * ((2.0 * u1 - 1.0) - (2.0 * u2 - 1.0)) * a.lo_ppm * 1e-6;
    const double ph = 2.0 * 3.14159265358979323846 * (u3 + f * static_cast<double>(i) / a.fs);
    double zr = yr, zi = yi;
    if (a.carrier) {
        double sn, cs;
        sincos(ph, &sn, &cs);
        zr = yr * cs - yi * sn;
        zi = yr * sn + yi * cs;
    }
    if (a.noise_sigma > 0.0) {
        uint64_t h = a.seed ^ (gs << 40) ^ static_cast<uint64_t>(i) ^ 0xA5A5A5A5ULL;
        const double n1 = 1.0 - u01(splitmix64(h));
        const double n2 = 1.0 - u01(splitmix64(h));
        const double mag = sqrt(-2.0 * log(n1)) * a.noise_sigma;
        zr += mag * cos(2.0 * 3.14159265358979323846 * n2);
        zi += mag * sin(2.0 * 3.14159265358979323846 * n2);
    }
    float *o = a.iq + s * a.stride + 2 * i;
    o[0] = static_cast<float>(zr);
    o[1] = static_cast<float>(zi);
}

thread_local std::string g_synth_err;

}  // namespace

extern "C" {

void qpsk_synth_params_init(qpsk_synth_params *p, int32_t sample_rate, int32_t symbol_rate) {
    std::memset(p, 0, sizeof(*p));
    p->sample_rate = sample_rate;
    p->symbol_rate = symbol_rate;
    p->rrc_alpha = static_cast<double>(0.4f);     // testAtDataLevel.cs:18
    p->rrc_span = 8;
    p->differential = 1;
    p->seed = 0x5159534BULL;
    p->lo_ppm = 1.0;                                // testAtDataLevel.cs:27-28
    p->cfo_hz = 0.0;
    p->multipath = 0;
    p->esn0_db = 1000.0;
}

int qpsk_synth_generate(const qpsk_synth_params *p, int32_t device, void *hip_stream,
                        int32_t n_streams, int64_t n_samples, float *iq_dev, int64_t stride_floats,
                        uint8_t *tx_bits_dev, int64_t bits_stride_bytes) {
    if (!p || !iq_dev) return QPSK_ERR_ARGUMENT_NULL;
    if (n_streams <= 0 || n_samples <= 0 || stride_floats < 2 * n_samples) return QPSK_ERR_ARGUMENT;
    if (p->symbol_rate <= 0 || p->sample_rate < p->symbol_rate) return QPSK_ERR_OUT_OF_RANGE;
    const int sps = p->sample_rate / p->symbol_rate;                  // QPSKModulator.cs:115
    std::vector<double> h = qpsk::rrc_coefficients(static_cast<double>(p->rrc_span), p->rrc_alpha,
                                                   p->sample_rate, p->symbol_rate);
    if (h.empty()) return QPSK_ERR_ARGUMENT;
    const int T = static_cast<int>(h.size());
    Pulse pulse{};
    // multipath [1, 0.25 e^{j0.7}, 0.1 e^{-j1.9}, 0.05] (sample spaced) folded into the pulse
    const double mr[4] = {1.0, 0.25 * std::cos(0.7), 0.1 * std::cos(-1.9), 0.05};
    const double mi[4] = {0.0, 0.25 * std::sin(0.7), 0.1 * std::sin(-1.9), 0.0};
    const int M = p->multipath ? 4 : 1;
    const int G = T + M - 1;
    if (G > 300) return QPSK_ERR_ARGUMENT;
    for (int k = 0; k < G; ++k) {
        double re = 0, im = 0;
        for (int j = 0; j < M; ++j) {
            const int t = k - j;
            if (t < 0 || t >= T) continue;
            const double hv = static_cast<double>(static_cast<float>(h[t]));   // float taps (:448-458)
            re += mr[j] * hv;
            im += mi[j] * hv;
        }
        pulse.re[k] = re;
        pulse.im[k] = im;
    }
    SynthArgs a{};
    a.S = n_streams;
    a.n = n_samples;
    a.sps = sps;
    a.mid = (T - 1) / 2;
    a.G = G;
    a.nsym = (n_samples + a.mid) / sps + 2;
    a.seed = p->seed;
    a.s0 = p->first_stream;
    a.cfo_hz = p->cfo_hz;
    a.lo_ppm = p->lo_ppm;
    a.lo_hz = 100e6;
    a.fs = static_cast<double>(p->sample_rate);
    // Es = 1 per symbol (unit-energy RRC, |sym| = 1): per-sample complex N0 = 1/EsN0
    a.noise_sigma = p->esn0_db < 200.0 ? std::sqrt(0.5 * std::pow(10.0, -p->esn0_db / 10.0)) : 0.0;
    a.differential = p->differential;
    a.carrier = (p->lo_ppm > 0.0 || p->cfo_hz > 0.0) ? 1 : 0;
    a.bits = tx_bits_dev;
    a.bits_stride = bits_stride_bytes;
    a.iq = iq_dev;
    a.stride = stride_floats;
    if (tx_bits_dev && bits_stride_bytes * 8 < 2 * a.nsym) return QPSK_ERR_ARGUMENT;
    if (hipSetDevice(device) != hipSuccess) return QPSK_ERR_DEVICE;
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    if (hipMalloc(reinterpret_cast<void **>(&a.quad), static_cast<size_t>(n_streams) * a.nsym) != hipSuccess)
        return QPSK_ERR_DEVICE;
    hipLaunchKernelGGL(synth_symbols_kernel, dim3((n_streams + 63) / 64), dim3(64), 0, st, a);
    dim3 grid(static_cast<unsigned>((n_samples + 255) / 256), static_cast<unsigned>(n_streams));
    hipLaunchKernelGGL(synth_samples_kernel, grid, dim3(256), 0, st, a, pulse);
    hipError_t e = hipStreamSynchronize(st);
    hipFree(a.quad);
    return e == hipSuccess ? QPSK_OK : QPSK_ERR_DEVICE;
}

}  // extern "C"
