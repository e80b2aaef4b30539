// qpsk_mod.hip -- the reference's QPSKModulator (QPSKModulator.cs:18-167) behind
// the C ABI, batched: one handle = the constructor (RRC taps, TSC, differential
// flag), one call = Modulate / ModulateBytes on S independent bit strings.
//
//   mod_symbols_kernel  one lane per stream: TSC + payload dibits -> symbols,
//                       differential (DibitToDelta :92-102, sym = prev * delta in
//                       float, reference (1/sqrt2)(1+j)) or direct (:140-144).
//                       The symbol of every dibit is +-InvSqrt2 on both axes,
//                       exactly, so it is kept as a 2-bit quadrant.
//   mod_samples_kernel  one thread per output sample: the impulse train (symbol
//                       d at delay + d*sps, :129-152) filtered by the float RRC
//                       taps in double, summed tap by tap in ascending tap
//                       order and rounded to float once -- the oracle's
//                       restatement of fftFilter (FIRFilter.cs:96-141; MathNet's
//                       FFT itself is absent here).
//
// Not the demodulation hot path: it generates transmit baseband on the GPU the
// way the reference's TX does.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "qpsk_demod.h"
#include "qpsk_design.h"

namespace qpsk {
int set_last_error(int code, const std::string &msg);
}

struct qpsk_mod {
    qpsk_mod_params p{};
    int T = 0;
    int sps = 0;
    int delay = 0;
    std::string tsc;           // "" = none (string.IsNullOrWhiteSpace)
    float *d_taps = nullptr;   // (float) RRC taps, T
    uint8_t *d_tsc = nullptr;  // TSC as packed bits
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // per-call device staging (grown as needed)
    uint8_t *d_quad = nullptr;
    size_t quad_bytes = 0;
    uint8_t *d_bits = nullptr;
    size_t bits_bytes = 0;
    int64_t *d_nbits = nullptr;
    int nbits_cap = 0;
    float *d_out = nullptr;
    size_t out_bytes = 0;
};

namespace {

using qpsk::set_last_error;

#define MOD_HIP_TRY(expr)                                                                      \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return set_last_error(QPSK_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

constexpr float kInvSqrt2 = 0.7071067811865475f;   // QPSKModulator.cs:36

struct ModArgs {
    int S;
    const uint8_t *bits;       // [S][bits_stride] packed MSB-first payload bits
    int64_t bits_stride;
    const int64_t *n_bits;     // [S]
    const uint8_t *tsc;        // packed TSC bits (prepended)
    int tsc_len;
    int differential;
    uint8_t *quad;             // [S][quad_stride] symbol quadrants
    int64_t quad_stride;
    int sps, delay, T;
    int pulse;
    const float *taps;
    float *out;                // [S][out_stride] interleaved
    int64_t out_stride;        // floats
    int64_t total_max;         // complex samples of the longest row
};

__device__ __forceinline__ int bit_at(const uint8_t *row, int64_t i) {
    return (row[i >> 3] >> (7 - (i & 7))) & 1;
}

// quadrant k <-> (+-InvSqrt2, +-InvSqrt2): 0 (+,+), 1 (-,+), 2 (-,-), 3 (+,-)
__global__ void mod_symbols_kernel(ModArgs a) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= a.S) return;
    const uint8_t *row = a.bits + s * a.bits_stride;
    const int64_t nbits = a.tsc_len + a.n_bits[s];
    const int64_t nd = nbits >> 1;   // "must have pairs of bits" (:113)
    uint8_t *q = a.quad + s * a.quad_stride;
    auto bit = [&](int64_t i) { return i < a.tsc_len ? bit_at(a.tsc, i) : bit_at(row, i - a.tsc_len); };
    int quad = 0;                    // the differential reference (1/sqrt2)(1+j)
    for (int64_t d = 0; d < nd; ++d) {
        const int bi = bit(2 * d), bq = bit(2 * d + 1);
        if (a.differential) {
            // DibitToDelta: 00 -> +1, 01 -> +j, 11 -> -1, 10 -> -j, i.e. a rotation
            // by 0, 1, 2, 3 quarter turns; prev * delta of +-InvSqrt2 components
            // with a unit axis phasor is exact in float
            const int rot = bi == 0 ? (bq == 0 ? 0 : 1) : (bq == 1 ? 2 : 3);
            quad = (quad + rot) & 3;
            q[d] = static_cast<uint8_t>(quad);
        } else {
            // symI = bi == 0 ? -InvSqrt2 : InvSqrt2, symQ likewise with bq
            q[d] = static_cast<uint8_t>(bi ? (bq ? 0 : 3) : (bq ? 1 : 2));
        }
    }
}

__global__ void mod_samples_kernel(ModArgs a) {
    const int s = blockIdx.y;
    const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t nd = (a.tsc_len + a.n_bits[s]) >> 1;
    const int64_t base_c = a.delay + nd * a.sps;
    const int64_t total = nd == 0 ? 0 : (a.pulse ? base_c + a.delay : base_c);
    if (i >= total) return;
    const uint8_t *q = a.quad + s * a.quad_stride;
    const float si[4] = {kInvSqrt2, -kInvSqrt2, -kInvSqrt2, kInvSqrt2};
    const float sq[4] = {kInvSqrt2, kInvSqrt2, -kInvSqrt2, -kInvSqrt2};
    float *o = a.out + s * a.out_stride + 2 * i;
    if (!a.pulse) {
        // the impulse train itself (:160-161)
        const int64_t r = i - a.delay;
        float vi = 0.f, vq = 0.f;
        if (r >= 0 && r % a.sps == 0 && r / a.sps < nd) {
            vi = si[q[r / a.sps]];
            vq = sq[q[r / a.sps]];
        }
        o[0] = vi;
        o[1] = vq;
        return;
    }
    // y[i] = sum_m taps[m] * up[T-1+i-m], m ascending; up[j] holds symbol d at
    // j = delay + d*sps (zeros elsewhere add nothing), fftFilter's slice at T-1
    double ar = 0.0, ai = 0.0;
    const int64_t top = a.T - 1 + i - a.delay;      // = m + d*sps for the tap m of symbol d
    // m ascending <=> d descending; m = top - d*sps in [0, T) and d in [0, nd)
    int64_t dhi = top / a.sps;                     // smallest m >= 0 ... largest d
    if (dhi > nd - 1) dhi = nd - 1;
    for (int64_t d = dhi; d >= 0; --d) {
        const int64_t m = top - d * a.sps;
        if (m >= a.T) break;
        const int k = q[d];
        const double h = static_cast<double>(a.taps[m]);
        ar += h * static_cast<double>(si[k]);
        ai += h * static_cast<double>(sq[k]);
    }
    o[0] = static_cast<float>(ar);
    o[1] = static_cast<float>(ai);
}

template <typename T>
int grow(T **p, size_t *have, size_t need_bytes) {
    if (need_bytes <= *have) return QPSK_OK;
    hipFree(*p);
    *p = nullptr;
    *have = 0;
    if (hipMalloc(reinterpret_cast<void **>(p), need_bytes) != hipSuccess)
        return set_last_error(QPSK_ERR_DEVICE, "hipMalloc (modulator staging)");
    *have = need_bytes;
    return QPSK_OK;
}

bool blank(const char *s) {
    if (!s) return true;
    for (; *s; ++s)
        if (!(*s == ' ' || (*s >= '\t' && *s <= '\r'))) return false;
    return true;
}

int64_t out_complex(const qpsk_mod *m, int64_t n_bits, int pulse) {
    const int64_t nd = (static_cast<int64_t>(m->tsc.size()) + std::max<int64_t>(0, n_bits)) >> 1;
    if (nd == 0) return 0;
    const int64_t base_c = m->delay + nd * m->sps;
    return pulse ? base_c + m->delay : base_c;
}

}  // namespace

extern "C" {

void qpsk_mod_params_init(qpsk_mod_params *p, int32_t sample_rate, int32_t symbol_rate) {
    std::memset(p, 0, sizeof(*p));
    p->sample_rate = sample_rate;
    p->symbol_rate = symbol_rate;
    p->rrc_alpha = 0.9;          // QPSKModulator.cs:18-24 defaults
    p->rrc_span = 6;
    p->differential = 1;
    p->device = 0;
}

int qpsk_mod_create(const qpsk_mod_params *p, const char *tsc, qpsk_mod **out) {
    if (!p || !out) return set_last_error(QPSK_ERR_ARGUMENT_NULL, "null argument");
    *out = nullptr;
    if (p->symbol_rate <= 0) return set_last_error(QPSK_ERR_OUT_OF_RANGE, "SymbolRate must be positive");
    if (tsc && !blank(tsc))
        for (const char *c = tsc; *c; ++c)
            if (*c != '0' && *c != '1') return set_last_error(QPSK_ERR_ARGUMENT, "tsc must be a '0'/'1' string");
    std::vector<double> h = qpsk::rrc_coefficients(static_cast<double>(p->rrc_span), p->rrc_alpha,
                                                   p->sample_rate, p->symbol_rate);
    if (h.empty()) return set_last_error(QPSK_ERR_ARGUMENT, "RRC design failed");
    auto *m = new qpsk_mod();
    m->p = *p;
    m->T = static_cast<int>(h.size());
    m->sps = p->sample_rate / p->symbol_rate;                  // :115 (integer division)
    m->delay = (m->T - 1) / 2;                                  // :119
    m->tsc = blank(tsc) ? std::string() : std::string(tsc);    // :26
    std::vector<float> tf(m->T);
    for (int k = 0; k < m->T; ++k) tf[k] = static_cast<float>(h[k]);   // ToInterleavedIQRealTapsStatic
    std::vector<uint8_t> tb((m->tsc.size() + 7) / 8 + 1, 0);
    for (size_t i = 0; i < m->tsc.size(); ++i)
        if (m->tsc[i] == '1') tb[i >> 3] |= static_cast<uint8_t>(0x80u >> (i & 7));
    if (hipSetDevice(p->device) != hipSuccess || hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(reinterpret_cast<void **>(&m->d_taps), m->T * sizeof(float)) != hipSuccess ||
        hipMalloc(reinterpret_cast<void **>(&m->d_tsc), tb.size()) != hipSuccess ||
        hipMemcpy(m->d_taps, tf.data(), m->T * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(m->d_tsc, tb.data(), tb.size(), hipMemcpyHostToDevice) != hipSuccess) {
        qpsk_mod_destroy(m);
        return set_last_error(QPSK_ERR_DEVICE, "modulator device set-up failed (no GPU?)");
    }
    m->own_stream = true;
    *out = m;
    return QPSK_OK;
}

int qpsk_mod_destroy(qpsk_mod *m) {
    if (!m) return QPSK_OK;
    if (m->stream) hipStreamSynchronize(m->stream);
    hipFree(m->d_taps);
    hipFree(m->d_tsc);
    hipFree(m->d_quad);
    hipFree(m->d_bits);
    hipFree(m->d_nbits);
    hipFree(m->d_out);
    if (m->own_stream && m->stream) hipStreamDestroy(m->stream);
    delete m;
    return QPSK_OK;
}

int qpsk_mod_set_stream(qpsk_mod *m, void *hip_stream) {
    if (!m) return set_last_error(QPSK_ERR_ARGUMENT_NULL, "null handle");
    MOD_HIP_TRY(hipStreamSynchronize(m->stream));
    if (hip_stream) {
        if (m->own_stream) hipStreamDestroy(m->stream);
        m->stream = static_cast<hipStream_t>(hip_stream);
        m->own_stream = false;
    } else if (!m->own_stream) {
        MOD_HIP_TRY(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
        m->own_stream = true;
    }
    return QPSK_OK;
}

int64_t qpsk_mod_output_floats(const qpsk_mod *m, int64_t n_bits, int32_t pulse_shaping) {
    if (!m) return 0;
    return 2 * out_complex(m, n_bits, pulse_shaping != 0);
}

int qpsk_mod_modulate(qpsk_mod *m, int32_t n_streams, const uint8_t *bits, int64_t bits_stride_bytes,
                      const int64_t *n_bits, int32_t pulse_shaping, int32_t mem, float *out,
                      int64_t out_stride_floats, int64_t *n_out_floats) {
    if (!m) return set_last_error(QPSK_ERR_ARGUMENT_NULL, "null handle");
    if (n_streams <= 0) return set_last_error(QPSK_ERR_ARGUMENT, "n_streams must be positive");
    if (!n_bits || !out || !n_out_floats) return set_last_error(QPSK_ERR_ARGUMENT_NULL, "data is null");
    if (mem != QPSK_MEM_HOST && mem != QPSK_MEM_DEVICE) return set_last_error(QPSK_ERR_ARGUMENT, "unknown mem");
    const int S = n_streams;
    const bool host = mem == QPSK_MEM_HOST;
    std::vector<int64_t> nb(S);
    if (host) std::memcpy(nb.data(), n_bits, S * sizeof(int64_t));
    else MOD_HIP_TRY(hipMemcpy(nb.data(), n_bits, S * sizeof(int64_t), hipMemcpyDeviceToHost));
    int64_t nb_max = 0, tot_max = 0;
    for (int s = 0; s < S; ++s) {
        if (nb[s] < 0) return set_last_error(QPSK_ERR_ARGUMENT, "negative bit count");
        nb_max = std::max(nb_max, nb[s]);
        tot_max = std::max(tot_max, out_complex(m, nb[s], pulse_shaping != 0));
    }
    if (nb_max > 0 && (!bits || bits_stride_bytes < (nb_max + 7) / 8))
        return set_last_error(bits ? QPSK_ERR_ARGUMENT : QPSK_ERR_ARGUMENT_NULL, "bit rows too short");
    if (out_stride_floats < 2 * tot_max) return set_last_error(QPSK_ERR_ARGUMENT, "out_stride_floats too small");
    MOD_HIP_TRY(hipSetDevice(m->p.device));
    hipStream_t st = m->stream;
    const int64_t nd_max = (static_cast<int64_t>(m->tsc.size()) + nb_max) / 2;
    int rc;
    ModArgs a{};
    a.S = S;
    a.bits = bits;
    a.bits_stride = bits_stride_bytes;
    a.n_bits = n_bits;
    a.out = out;
    a.out_stride = out_stride_floats;
    if (host) {
        const size_t brow = static_cast<size_t>((nb_max + 7) / 8 + 1);
        if ((rc = grow(&m->d_bits, &m->bits_bytes, S * brow))) return rc;
        if (nb_max > 0)
            MOD_HIP_TRY(hipMemcpy2DAsync(m->d_bits, brow, bits, bits_stride_bytes, (nb_max + 7) / 8, S,
                                         hipMemcpyHostToDevice, st));
        if (S > m->nbits_cap) {
            hipFree(m->d_nbits);
            m->d_nbits = nullptr;
            m->nbits_cap = 0;
            if (hipMalloc(reinterpret_cast<void **>(&m->d_nbits), S * sizeof(int64_t)) != hipSuccess)
                return set_last_error(QPSK_ERR_DEVICE, "hipMalloc");
            m->nbits_cap = S;
        }
        MOD_HIP_TRY(hipMemcpyAsync(m->d_nbits, nb.data(), S * sizeof(int64_t), hipMemcpyHostToDevice, st));
        const size_t orow = static_cast<size_t>(2 * std::max<int64_t>(tot_max, 1));
        if ((rc = grow(&m->d_out, &m->out_bytes, S * orow * sizeof(float)))) return rc;
        a.bits = m->d_bits;
        a.bits_stride = static_cast<int64_t>(brow);
        a.n_bits = m->d_nbits;
        a.out = m->d_out;
        a.out_stride = static_cast<int64_t>(orow);
    }
    if ((rc = grow(&m->d_quad, &m->quad_bytes, static_cast<size_t>(S) * std::max<int64_t>(nd_max, 1)))) return rc;
    a.tsc = m->d_tsc;
    a.tsc_len = static_cast<int>(m->tsc.size());
    a.differential = m->p.differential;
    a.quad = m->d_quad;
    a.quad_stride = std::max<int64_t>(nd_max, 1);
    a.sps = m->sps;
    a.delay = m->delay;
    a.T = m->T;
    a.pulse = pulse_shaping != 0;
    a.taps = m->d_taps;
    a.total_max = tot_max;
    if (tot_max > 0) {
        hipLaunchKernelGGL(mod_symbols_kernel, dim3((S + 63) / 64), dim3(64), 0, st, a);
        dim3 grid(static_cast<unsigned>((tot_max + 255) / 256), static_cast<unsigned>(S));
        hipLaunchKernelGGL(mod_samples_kernel, grid, dim3(256), 0, st, a);
        MOD_HIP_TRY(hipGetLastError());
    }
    std::vector<int64_t> nout(S);
    for (int s = 0; s < S; ++s) nout[s] = 2 * out_complex(m, nb[s], pulse_shaping != 0);
    if (host) {
        if (tot_max > 0)
            MOD_HIP_TRY(hipMemcpy2DAsync(out, out_stride_floats * sizeof(float), a.out, a.out_stride * sizeof(float),
                                         2 * tot_max * sizeof(float), S, hipMemcpyDeviceToHost, st));
        MOD_HIP_TRY(hipStreamSynchronize(st));
        std::memcpy(n_out_floats, nout.data(), S * sizeof(int64_t));
    } else {
        MOD_HIP_TRY(hipMemcpyAsync(n_out_floats, nout.data(), S * sizeof(int64_t), hipMemcpyHostToDevice, st));
        MOD_HIP_TRY(hipStreamSynchronize(st));   // nout is a host temporary
    }
    return QPSK_OK;
}

int qpsk_mod_modulate_bytes(qpsk_mod *m, int32_t n_streams, const uint8_t *payload, int64_t payload_stride,
                            const int64_t *n_payload, const uint8_t *start_marker, int32_t n_start,
                            const uint8_t *end_marker, int32_t n_end, int32_t pulse_shaping, float *out,
                            int64_t out_stride_floats, int64_t *n_out_floats) {
    if (!m) return set_last_error(QPSK_ERR_ARGUMENT_NULL, "null handle");
    if (n_start <= 0 || !start_marker) return set_last_error(QPSK_ERR_ARGUMENT, "startMarker cannot be empty.");
    if (n_end <= 0 || !end_marker) return set_last_error(QPSK_ERR_ARGUMENT, "endMarker cannot be empty.");
    if (n_streams <= 0 || !n_payload) return set_last_error(QPSK_ERR_ARGUMENT_NULL, "payload is null");
    // frame START + payload + END (QPSKModulator.cs:54-72), bits MSB-first
    // (BitPacker.BytesToBitString, HelperFunctions.cs:14-29)
    const int S = n_streams;
    int64_t pmax = 0;
    for (int s = 0; s < S; ++s) {
        if (n_payload[s] < 0) return set_last_error(QPSK_ERR_ARGUMENT, "negative payload length");
        pmax = std::max(pmax, n_payload[s]);
    }
    if (pmax > 0 && (!payload || payload_stride < pmax)) return set_last_error(QPSK_ERR_ARGUMENT, "payload rows too short");
    const int64_t row = n_start + pmax + n_end;
    std::vector<uint8_t> framed(static_cast<size_t>(S) * row);
    std::vector<int64_t> nb(S);
    for (int s = 0; s < S; ++s) {
        uint8_t *f = framed.data() + s * row;
        std::memcpy(f, start_marker, n_start);
        if (n_payload[s]) std::memcpy(f + n_start, payload + s * payload_stride, n_payload[s]);
        std::memcpy(f + n_start + n_payload[s], end_marker, n_end);
        nb[s] = 8 * (n_start + n_payload[s] + n_end);
    }
    return qpsk_mod_modulate(m, S, framed.data(), row, nb.data(), pulse_shaping, QPSK_MEM_HOST, out,
                             out_stride_floats, n_out_floats);
}

}  // extern "C"
