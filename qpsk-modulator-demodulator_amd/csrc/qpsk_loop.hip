// qpsk_loop.hip -- symbol sync + carrier recovery + decode on gfx950.
//
// MuellerMuller.Process (MuellerMuller.cs:52-190), CostasLoopQpsk.Process
// (CostasLoopQpsk.cs:63-92), the hard decision, differential decode and
// MSB-first bit packing of QPSKDeModulator.DeModulate (QPSKDeModulator.cs:
// 364-408).  Both loops are serial recurrences per stream, so a stream's work
// cannot be spread over lanes; measured on MI355X (tools/loop_latency.hip) one
// wave issues a dependent FP64 op every ~7.5 cycles and the per-symbol chains
// are issue/latency-bound, so the lever is to give each stage of a stream its
// OWN wave (its own SIMD issue port) and keep memory off the chains:
//
//   workgroup = 4 waves, SPW streams (one lane each):
//     wave 0  loader  HBM -> LDS ring of matched-filter samples with
//                     global_load_lds_dwordx4 (no VGPR staging), 2 rounds ahead
//     wave 1  M&M     timing recovery: ring -> interpolated symbols (round r)
//     wave 2  Costas  carrier recovery on the symbols of round r-1 -> rotated
//     wave 3  decode  decision + differential decode + bit packing + stores of
//                     the rotated symbols of round r-2
//   round r = samples [r*kB, (r+1)*kB) of every stream's queue; one raw
//   s_barrier per round hands every ring slot one stage forward.
//
// The stages never feed back into an earlier one (Costas does not drive the
// timing loop) and symbols flow in order, so the outputs are exactly the
// reference's.
//
// The M&M queue of a stream (MuellerMuller.cs:32-36) = R retained samples of
// the previous call (carry) followed by this call's n MF samples; logical index
// i of the reference maps to physical index p = i + (R & 1), so physical 0 is
// 16-byte aligned in the MF buffer (carry placed at kMfPrefix - R).
//
// -ffp-contract=off: every float/double op rounds as the reference C#.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "qpsk_kernels.h"
#include "qpsk_sincos.h"

namespace qpsk {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

#ifdef QPSK_LOOP_STAMPS
#define STAMP(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#define ACC(acc, t0) acc += __builtin_amdgcn_s_memtime() - (t0)
#else
#define STAMP(v)
#define ACC(acc, t0)
#endif

constexpr int kB = 64;            // samples per round per stream
constexpr int kRing = 4 * kB;     // per-stream sample ring (4 rounds): index = p & (kRing-1)
constexpr int kMir = 4;           // mirror of the ring's last samples in front of it, so the
                                  // 4 interpolation taps are always contiguous in LDS
constexpr int kRowS = kMir + kRing;   // per-stream LDS row: [mirror 4][ring 256]
constexpr int kSymCap = 80;       // symbols per round per stream: <= 67 / (sps - 0.1) + 1, sps >= 1

__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int w = __shfl_xor(v, o, 64);
        v = w > v ? w : v;
    }
    return v;
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), l);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32), l);
    return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
}

// carry (retained queue of the previous call) -> MF buffer prefix
__global__ void carry_prefix_kernel(LoopArgs a) {
    const int s = blockIdx.x;
    if (s >= a.S) return;
    const int R = a.state[s].carry_n;
    const f2 *c = reinterpret_cast<const f2 *>(a.carry) + static_cast<int64_t>(s) * kCarryMax;
    f2 *mf = reinterpret_cast<f2 *>(a.mf) + s * a.mf_stride + kMfPrefix - R;
    for (int i = threadIdx.x; i < R; i += blockDim.x) mf[i] = c[i];
}

template <int SPW>
struct LoopLds {
    f2 mf[SPW * kRowS];            // sample ring   [stream][mirror | 4 rounds x kB]
    f2 sym[2 * SPW * kSymCap];     // M&M -> Costas [slot][stream][kSymCap]
    f2 rot[2 * SPW * kSymCap];     // Costas -> decode
    int cnt[4 * SPW];              // symbols produced by the M&M in round r: cnt[r & 3]
};

template <int MODE, bool DIFF, bool SYMS, int SPW>
__global__ __launch_bounds__(256) void loop_kernel(LoopArgs a, LoopParams P) {
    // one LDS object only: a second __shared__ object would make hipcc drain the
    // loader's LDS-DMA before touching it (cdna_hip_programming.md §5)
    __shared__ LoopLds<SPW> L;

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int s = blockIdx.x * SPW + lane;
    const bool valid = lane < SPW && s < a.S;

    // ---- per-stream queue geometry (every wave: lane l <-> stream blk*SPW + l)
    int n = 0, cnt = 0, R = 0, d = 0;
    if (valid) {
        n = static_cast<int>(a.lengths ? a.lengths[s] : a.n);
        R = a.state[s].carry_n;
        d = R & 1;
        cnt = R + d + n;
        // DeModulate with an empty span returns before touching any state (:350-351)
        if (MODE == kModeDemodulate && n == 0) cnt = 0;
    }
    const int NR = (wave_max_i32(cnt) + kB - 1) / kB;
    const bool mine = valid && cnt > 0;

    if (wave == 0) {
        // ============================================================ loader
        // one glds instruction = 32 lanes x 16 B = one stream's round (512 B)
        const int64_t org = valid ? s * a.mf_stride + kMfPrefix - R - d : 0;
        const int c2 = 2 * (lane & 31);
        const f2 *mf = reinterpret_cast<const f2 *>(a.mf);
        const bool lo_half = lane < 32;
        auto issue = [&](int r) {
            const int roff = (r & 3) * kB;
#pragma unroll 4
            for (int j = 0; j < SPW; ++j) {
                const int c = __builtin_amdgcn_readlane(cnt, j);
                const int64_t o = readlane64(org, j);
                int p = r * kB + c2;
                // past the stream's end: read a harmless in-row pair (never used);
                // a pair straddling the end reads one sample of row slack
                if (p >= c) p = 0;
                if (lo_half)
                    __builtin_amdgcn_global_load_lds((glb_void_t *)(mf + o + p),
                                                     (lds_void_t *)(L.mf + j * kRowS + kMir + roff), 16, 0, 0);
            }
        };
#ifdef QPSK_LOOP_STAMPS
        unsigned long long t_wait = 0, t_bar = 0;
#endif
        if (NR > 0) issue(0);
        if (NR > 1) issue(1);
        for (int r = 0; r <= NR + 1; ++r) {
            STAMP(ta);
            if (r + 1 < NR) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(SPW) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            ACC(t_wait, ta);
            STAMP(tb);
            __builtin_amdgcn_s_barrier();
            ACC(t_bar, tb);
            if (r + 2 < NR) issue(r + 2);
        }
#ifdef QPSK_LOOP_STAMPS
        if (a.probe && lane == 0) {
            a.probe[blockIdx.x * 8 + 0] = t_wait;
            a.probe[blockIdx.x * 8 + 1] = t_bar;
        }
#endif
        return;
    }

    if (wave == 1) {
        // ============================================================ M&M
        StreamState st;
        if (mine) st = a.state[s];
        int base = mine ? st.base + d : 0;          // physical baseIndex
        double mu = st.mu, integ = st.integ;
        float psi = st.psi, psq = st.psq, pdi = st.pdi, pdq = st.pdq;
        int has_prev = mine ? st.has_prev : 1;
        const double sps = P.sps, kp = P.kp, ki = P.ki;
        const double dd = static_cast<double>(d);
        const int cap = n;                          // output span = 2n floats (QPSKDeModulator.cs:366)
        int nsym = 0;
        bool stop = !mine;                          // capacity reached (MuellerMuller.cs:101-102)
        f2 *row = L.mf + lane * kRowS;
        // taps x[b-1..b+2] of physical index b: contiguous thanks to the mirror
        auto taps = [&](int b) -> const f2 * { return row + kMir - 3 + ((b + 2) & (kRing - 1)); };
        // the TED reuses the previous symbol widened to double (MuellerMuller.cs:78-80)
        double psid = psi, psqd = psq;
#ifdef QPSK_LOOP_STAMPS
        unsigned long long c_bar = 0, c_loop = 0, c_iters = 0;
#endif
        for (int r = 0; r <= NR + 1; ++r) {
            STAMP(tb);
            __builtin_amdgcn_s_barrier();
            ACC(c_bar, tb);
            if (r >= NR) continue;
            STAMP(tl);
            if ((r & 3) == 0 && r > 0 && mine) {
                // mirror = last 4 samples of the ring (round r-1, already consumed)
                row[0] = row[kMir + kRing - 4]; row[1] = row[kMir + kRing - 3];
                row[2] = row[kMir + kRing - 2]; row[3] = row[kMir + kRing - 1];
            }
            const int rend = (r + 1) * kB < cnt ? (r + 1) * kB : cnt;
            f2 *out = L.sym + ((r & 1) * SPW + lane) * kSymCap;
            int kmax = stop ? 0 : (cap - nsym < kSymCap ? cap - nsym : kSymCap);
            int k = 0;
            const f2 *tp = taps(base);
            f2 xm1 = tp[0], x0 = tp[1], x1 = tp[2], x2 = tp[3];
            if (!has_prev && base + 2 < rend && kmax > 0) {
                // very first symbol of the stream: no TED, advance = sps (MuellerMuller.cs:93-97)
                const float t = static_cast<float>(mu);
                const float tm1 = t - 1.0f, tm2 = t - 2.0f, tp1 = t + 1.0f;
                const float cm1 = -(t * tm1 * tm2) * (1.0f / 6.0f);
                const float c0 = (tp1 * tm1 * tm2) * (1.0f / 2.0f);
                const float c1 = -(tp1 * t * tm2) * (1.0f / 2.0f);
                const float c2 = (tp1 * t * tm1) * (1.0f / 6.0f);
                const float ci = cm1 * xm1.x + c0 * x0.x + c1 * x1.x + c2 * x2.x;
                const float cq = cm1 * xm1.y + c0 * x0.y + c1 * x1.y + c2 * x2.y;
                has_prev = 1;
                out[k++] = f2{ci, cq};
                psi = ci; psq = cq;
                psid = ci; psqd = cq;
                pdi = ci >= 0.0f ? 1.0f : -1.0f;
                pdq = cq >= 0.0f ? 1.0f : -1.0f;
                const double nt = static_cast<double>(base - d) + mu + sps;
                const double fl = floor(nt);
                base = static_cast<int>(fl) + d;
                mu = nt - fl;
                tp = taps(base);
                xm1 = tp[0]; x0 = tp[1]; x1 = tp[2]; x2 = tp[3];
            }
            while (base + 2 < rend && k < kmax) {
                // CubicLagrange4 (MuellerMuller.cs:160-190), float
                const float t = static_cast<float>(mu);
                const float tm1 = t - 1.0f, tm2 = t - 2.0f, tp1 = t + 1.0f;
                const float cm1 = -(t * tm1 * tm2) * (1.0f / 6.0f);
                const float c0 = (tp1 * tm1 * tm2) * (1.0f / 2.0f);
                const float c1 = -(tp1 * t * tm2) * (1.0f / 2.0f);
                const float c2 = (tp1 * t * tm1) * (1.0f / 6.0f);
                const float ci = cm1 * xm1.x + c0 * x0.x + c1 * x1.x + c2 * x2.x;
                const float cq = cm1 * xm1.y + c0 * x0.y + c1 * x1.y + c2 * x2.y;
                // M&M TED (MuellerMuller.cs:78-80): decisions are +-1, so each
                // (double)d * x product is exactly +-x
                const double cid = ci, cqd = cq;
                const double t1 = (pdi >= 0.0f ? cid : -cid) + (pdq >= 0.0f ? cqd : -cqd);
                const double t2 = (ci >= 0.0f ? psid : -psid) + (cq >= 0.0f ? psqd : -psqd);
                const double e = t1 - t2;
                // PI filter, clamp, advance (MuellerMuller.cs:83-91)
                integ = integ + ki * e;
                double corr = kp * e + integ;
                corr = corr > 0.1 ? 0.1 : corr;
                corr = corr < -0.1 ? -0.1 : corr;
                const double adv = sps + corr;
                out[k++] = f2{ci, cq};
                psi = ci; psq = cq;
                psid = cid; psqd = cqd;
                pdi = ci >= 0.0f ? 1.0f : -1.0f;
                pdq = cq >= 0.0f ? 1.0f : -1.0f;
                const double nt = static_cast<double>(base - d) + mu + adv;   // :113-115
                const double fl = floor(nt);
                base = static_cast<int>(fl) + d;
                mu = nt - fl;
                tp = taps(base);
                xm1 = tp[0]; x0 = tp[1]; x1 = tp[2]; x2 = tp[3];
#ifdef QPSK_LOOP_STAMPS
                ++c_iters;
#endif
            }
            nsym += k;
            if (!stop && nsym >= cap && base + 2 < rend) {
                // MuellerMuller.cs:73-102: the symbol after the last one that fits
                // still runs the TED/PI update, then the call stops
                const float t = static_cast<float>(mu);
                const float tm1 = t - 1.0f, tm2 = t - 2.0f, tp1 = t + 1.0f;
                const float cm1 = -(t * tm1 * tm2) * (1.0f / 6.0f);
                const float c0 = (tp1 * tm1 * tm2) * (1.0f / 2.0f);
                const float c1 = -(tp1 * t * tm2) * (1.0f / 2.0f);
                const float c2 = (tp1 * t * tm1) * (1.0f / 6.0f);
                const float ci = cm1 * xm1.x + c0 * x0.x + c1 * x1.x + c2 * x2.x;
                const float cq = cm1 * xm1.y + c0 * x0.y + c1 * x1.y + c2 * x2.y;
                const float di = ci >= 0.0f ? 1.0f : -1.0f;
                const float dq = cq >= 0.0f ? 1.0f : -1.0f;
                if (has_prev) {
                    const double t1 = static_cast<double>(pdi) * ci + static_cast<double>(pdq) * cq;
                    const double t2 = static_cast<double>(di) * psi + static_cast<double>(dq) * psq;
                    integ += ki * (t1 - t2);
                }
                has_prev = 1;
                stop = true;
            }
            if (lane < SPW) L.cnt[(r & 3) * SPW + lane] = k;
            ACC(c_loop, tl);
        }
#ifdef QPSK_LOOP_STAMPS
        if (a.probe && lane == 0) {
            a.probe[blockIdx.x * 8 + 2] = c_bar;
            a.probe[blockIdx.x * 8 + 3] = c_loop;
            a.probe[blockIdx.x * 8 + 4] = c_iters;
            a.probe[blockIdx.x * 8 + 7] = NR;
        }
#endif
        if (!valid) return;
        if (!mine) {   // empty DeModulate call: nothing changes
            if (a.n_syms) a.n_syms[s] = 0;
            return;
        }
        if (a.n_syms) a.n_syms[s] = nsym;
        // drop consumed samples, keep the rest for the next call (MuellerMuller.cs:123-133)
        const int count = R + n;
        const int lbase = base - d;
        int consumed = lbase - 1 > 0 ? lbase - 1 : 0;
        const int keep_min = count - 3 > 0 ? count - 3 : 0;
        if (keep_min < consumed) consumed = keep_min;
        int keep = count - consumed;
        if (keep > kCarryMax) {
            atomicOr(&a.state[s].error, 1);
            consumed = count - kCarryMax;
            keep = kCarryMax;
        }
        const f2 *q = reinterpret_cast<const f2 *>(a.mf) + s * a.mf_stride + kMfPrefix - R;  // logical 0
        f2 *cw = reinterpret_cast<f2 *>(a.carry) + static_cast<int64_t>(s) * kCarryMax;
        for (int i = 0; i < keep; ++i) cw[i] = q[consumed + i];
        StreamState *g = a.state + s;
        g->base = lbase - consumed;
        g->carry_n = keep;
        g->mu = mu;
        g->integ = integ;
        g->psi = psi; g->psq = psq; g->pdi = pdi; g->pdq = pdq;
        g->has_prev = has_prev;
        return;
    }

    if (wave == 2) {
        // ============================================================ Costas
        double theta = 0.0, freq = 0.0;
        if (mine) {
            theta = a.state[s].theta;
            freq = a.state[s].freq;
        }
        const double ca = P.c_alpha, cb = P.c_beta;
        const double kTwoPi = 2.0 * 3.14159265358979311600;
        const double kPi = 3.14159265358979311600;
#ifdef QPSK_LOOP_STAMPS
        unsigned long long k_bar = 0, k_loop = 0;
#endif
        for (int r = 0; r <= NR + 1; ++r) {
            STAMP(tb);
            __builtin_amdgcn_s_barrier();
            ACC(k_bar, tb);
            if (r == 0 || r > NR) continue;
            STAMP(tl);
            const int slot = (r - 1) & 1;
            const int m = mine ? L.cnt[((r - 1) & 3) * SPW + lane] : 0;
            const f2 *in = L.sym + (slot * SPW + lane) * kSymCap;
            f2 *out = L.rot + (slot * SPW + lane) * kSymCap;
            f2 y = in[0];
            for (int k = 0; k < m; ++k) {
                const f2 yn = in[k + 1];   // next symbol, read under this one's chain
                // CostasLoopQpsk.cs:63-92: double NCO, float I/O
                double sn, cs;
                qpsk_sincos(theta, &sn, &cs);
                const double mi = static_cast<double>(y.x) * cs + static_cast<double>(y.y) * sn;
                const double mq = static_cast<double>(y.y) * cs - static_cast<double>(y.x) * sn;
                const float ri = static_cast<float>(mi), rq = static_cast<float>(mq);
                // (double)e * m with e = +-1 is exact: a sign flip gives the same number
                const double pe = (ri >= 0.0f ? mq : -mq) - (rq >= 0.0f ? mi : -mi);
                freq = freq + cb * pe;
                theta = theta + (freq + ca * pe);
                if (__builtin_expect(fabs(theta) > kPi, 0))        // CostasLoopQpsk.cs:89-91
                    theta = theta > kPi ? theta - kTwoPi : theta + kTwoPi;
                out[k] = f2{ri, rq};
                y = yn;
            }
            ACC(k_loop, tl);
        }
#ifdef QPSK_LOOP_STAMPS
        if (a.probe && lane == 0) {
            a.probe[blockIdx.x * 8 + 5] = k_bar;
            a.probe[blockIdx.x * 8 + 6] = k_loop;
        }
#endif
        if (mine) {
            a.state[s].theta = theta;
            a.state[s].freq = freq;
        }
        return;
    }

    // ================================================================ decode
    int diff_have = 0;
    float dpi = 0.f, dpq = 0.f;
    if (mine) {
        diff_have = a.state[s].diff_have;
        dpi = a.state[s].diff_pi;
        dpq = a.state[s].diff_pq;
    }
    uint32_t *bits = (MODE == kModeDemodulate && mine) ? a.bits + s * a.bits_stride_words : nullptr;
    f2 *syms = (SYMS && mine) ? reinterpret_cast<f2 *>(a.syms) + s * a.syms_stride : nullptr;
    uint32_t word = 0;
    int wbits = 0;
    int64_t widx = 0, nbits = 0, ncs = 0;
    int err = 0;
    for (int r = 0; r <= NR + 1; ++r) {
        __builtin_amdgcn_s_barrier();
        if (r < 2) continue;
        const int slot = (r - 2) & 1;
        const int m = mine ? L.cnt[((r - 2) & 3) * SPW + lane] : 0;
        const f2 *in = L.rot + (slot * SPW + lane) * kSymCap;
        for (int k = 0; k < m; ++k) {
            const f2 rr = in[k];
            if (SYMS) {
                if (ncs < a.syms_cap) syms[ncs] = rr;
                else err |= 2;
            }
            ++ncs;
            if (MODE == kModeDemodulate) {
                // decision + differential decode (QPSKDeModulator.cs:379-407, 304-337)
                const float ei = rr.x >= 0.0f ? 1.0f : -1.0f;
                const float eq = rr.y >= 0.0f ? 1.0f : -1.0f;
                uint32_t b2;
                bool emit = true;
                if (DIFF) {
                    const float del_i = ei * dpi + eq * dpq;
                    const float del_q = eq * dpi - ei * dpq;
                    emit = diff_have != 0;
                    diff_have = 1;
                    dpi = ei;
                    dpq = eq;
                    b2 = fabsf(del_i) >= fabsf(del_q) ? (del_i >= 0.0f ? 0u : 3u)
                                                      : (del_q >= 0.0f ? 1u : 2u);
                } else {
                    b2 = (ei < 0.0f ? 0u : 2u) | (eq < 0.0f ? 0u : 1u);
                }
                if (emit) {
                    word = (word << 2) | b2;
                    wbits += 2;
                    nbits += 2;
                    if (wbits == 32) {
                        if (widx < a.bits_cap_words) bits[widx] = __builtin_bswap32(word);
                        else err |= 2;
                        ++widx;
                        word = 0;
                        wbits = 0;
                    }
                }
            }
        }
    }
    if (!valid) return;
    if (!mine) {
        if (a.n_bits) a.n_bits[s] = 0;
        return;
    }
    if (MODE == kModeDemodulate && wbits > 0) {
        if (widx < a.bits_cap_words) bits[widx] = __builtin_bswap32(word << (32 - wbits));
        else err |= 2;
    }
    StreamState *g = a.state + s;
    if (MODE == kModeDemodulate) {
        g->diff_have = diff_have;
        g->diff_pi = dpi;
        g->diff_pq = dpq;
    }
    if (err) atomicOr(&g->error, err);
    if (a.n_bits) a.n_bits[s] = MODE == kModeDemodulate ? nbits : 0;
}

template <int SPW>
static void launch_loop_spw(const LoopArgs &a, const LoopParams &P, int mode, hipStream_t stream) {
    dim3 grid((a.S + SPW - 1) / SPW), block(256);
    const bool syms = a.syms != nullptr;
    const bool diff = P.differential != 0;
    if (mode == kModeConstellation)
        hipLaunchKernelGGL((loop_kernel<kModeConstellation, false, true, SPW>), grid, block, 0, stream, a, P);
    else if (diff && syms)
        hipLaunchKernelGGL((loop_kernel<kModeDemodulate, true, true, SPW>), grid, block, 0, stream, a, P);
    else if (diff)
        hipLaunchKernelGGL((loop_kernel<kModeDemodulate, true, false, SPW>), grid, block, 0, stream, a, P);
    else if (syms)
        hipLaunchKernelGGL((loop_kernel<kModeDemodulate, false, true, SPW>), grid, block, 0, stream, a, P);
    else
        hipLaunchKernelGGL((loop_kernel<kModeDemodulate, false, false, SPW>), grid, block, 0, stream, a, P);
}

void launch_loop(const LoopArgs &a, const LoopParams &P, int mode, int streams_per_block,
                 hipStream_t stream) {
    hipLaunchKernelGGL(carry_prefix_kernel, dim3(a.S), dim3(64), 0, stream, a);
    // the loop is latency-bound per stream and a wave's lanes are free, so
    // 32 streams per workgroup; measured faster than 16 even at S=256, where
    // only 8 CUs are busy (profiles/r01_loop_probe.txt)
    if (streams_per_block == 16)
        launch_loop_spw<16>(a, P, mode, stream);
    else
        launch_loop_spw<32>(a, P, mode, stream);
}

}  // namespace qpsk
