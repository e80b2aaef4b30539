// qpsk_loop.hip -- symbol sync + carrier recovery + decode on gfx950.
//
// MuellerMuller.Process (MuellerMuller.cs:52-190) fused with
// CostasLoopQpsk.Process (CostasLoopQpsk.cs:63-92), the hard decision,
// differential decode and MSB-first bit packing of QPSKDeModulator.DeModulate
// (QPSKDeModulator.cs:372-408).  The recurrences are serial per stream, so one
// lane owns one stream; the kernel is latency-bound, and its design goal is to
// keep HBM latency off each lane's dependency chain:
//
//   workgroup = 2 waves:
//     wave 0 (consumer): one lane per stream, runs the loops reading the
//             matched-filter samples from an LDS ring only;
//     wave 1 (loader):   streams each stream's samples HBM -> LDS with
//             global_load_lds_dwordx4 (no VGPR staging), two rounds ahead.
//   ring = kR rounds x SPW streams x kB samples (float2); round r holds the
//   samples [r*kB, (r+1)*kB) of every stream's queue ("physical" index, see
//   below).  Per round: loader waits for round r (counted vmcnt), one raw
//   s_barrier, issues round r+2 into the slot the consumer no longer needs;
//   the consumer runs every lane's symbols whose 4 interpolation taps lie below
//   the round end.
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

constexpr int kB = 64;    // samples per round per stream
constexpr int kR = 4;     // ring depth (rounds); loader runs 2 rounds ahead

__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t w = __shfl_xor(v, o, 64);
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

template <int MODE, bool DIFF, bool SYMS, int SPW>
__global__ __launch_bounds__(128) void loop_kernel(LoopArgs a, LoopParams P) {
    // the ring is the ONLY LDS object: a second one would make hipcc wait for
    // every outstanding LDS-DMA before touching it (cdna_hip_programming.md §5)
    __shared__ f2 ring[kR * SPW * kB];
    constexpr int kPerRound = SPW / 2;   // glds instructions per round (2 streams x 512 B each)

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int s = blockIdx.x * SPW + lane;
    const bool mine = (wave == 0) && lane < SPW && s < a.S;
    // both waves: lane l < SPW describes stream blockIdx.x*SPW + l

    // ---- per-stream queue geometry -------------------------------------
    int64_t n = 0, cnt = 0;
    int R = 0, d = 0;
    if (lane < SPW && s < a.S) {
        n = a.lengths ? a.lengths[s] : a.n;
        R = a.state[s].carry_n;
        d = R & 1;
        cnt = R + d + n;
        // DeModulate with an empty span returns before touching any state (:350-351)
        if (MODE == kModeDemodulate && n == 0) cnt = 0;
    }
    const int64_t org = (lane < SPW && s < a.S) ? s * a.mf_stride + kMfPrefix - R - d : 0;
    const int64_t maxc = wave_max_i64(cnt);
    const int NR = static_cast<int>((maxc + kB - 1) / kB);

    if (wave == 1) {
        // ------------------------------------------------------------ loader
        const int half = lane >> 5;          // which of the 2 streams of one instruction
        const int c2 = 2 * (lane & 31);      // first of the 2 samples this lane moves
        const f2 *mf = reinterpret_cast<const f2 *>(a.mf);
        auto issue = [&](int r) {
            f2 *slot = ring + (r & (kR - 1)) * SPW * kB;
#pragma unroll 4
            for (int j = 0; j < kPerRound; ++j) {
                // geometry of streams 2j, 2j+1 from their lanes (readlane: no LDS access)
                const int64_t c = half ? readlane64(cnt, 2 * j + 1) : readlane64(cnt, 2 * j);
                const int64_t o = half ? readlane64(org, 2 * j + 1) : readlane64(org, 2 * j);
                int64_t p = static_cast<int64_t>(r) * kB + c2;
                // past the stream's end: read a harmless in-row pair (never used);
                // a pair straddling the end reads one sample of row slack
                if (p >= c) p = 0;
                const f2 *src = mf + o + p;
                __builtin_amdgcn_global_load_lds((glb_void_t *)src,
                                                 (lds_void_t *)(slot + (2 * j) * kB), 16, 0, 0);
            }
        };
#ifdef QPSK_LOOP_STAMPS
        unsigned long long t_wait = 0, t_bar = 0, t_issue = 0;
#endif
        if (NR > 0) issue(0);
        if (NR > 1) issue(1);
        for (int r = 0; r < NR; ++r) {
            STAMP(ta);
            if (r + 1 < NR) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPerRound) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            ACC(t_wait, ta);
            STAMP(tb);
            __builtin_amdgcn_s_barrier();
            ACC(t_bar, tb);
            STAMP(tc);
            if (r + 2 < NR) issue(r + 2);
            ACC(t_issue, tc);
        }
#ifdef QPSK_LOOP_STAMPS
        if (a.probe && lane == 0) {
            a.probe[blockIdx.x * 8 + 0] = t_wait;
            a.probe[blockIdx.x * 8 + 1] = t_bar;
            a.probe[blockIdx.x * 8 + 2] = t_issue;
        }
#endif
        return;
    }

    // -------------------------------------------------------------- consumer
    // Software-pipelined: iteration k runs Costas + decode on the symbol the
    // M&M produced in iteration k-1 AND the M&M step for the next symbol; the
    // two recurrences are independent (Costas never feeds the timing loop), so
    // their dependency chains overlap.  Both halves are straight-line code whose
    // state updates are committed with selects (no divergent branches inside an
    // iteration).  Order of results is exactly the reference's: the M&M emits
    // symbols in order, Costas consumes them in order.
    StreamState st;
    if (mine) st = a.state[s];
    int64_t base = mine ? st.base + d : 0;     // physical baseIndex
    double mu = st.mu, integ = st.integ;
    float psi = st.psi, psq = st.psq, pdi = st.pdi, pdq = st.pdq;
    int has_prev = st.has_prev;
    double theta = st.theta, freq = st.freq;
    int diff_have = st.diff_have;
    float dpi = st.diff_pi, dpq = st.diff_pq;
    int err = st.error;
    const double sps = P.sps, kp = P.kp, ki = P.ki, ca = P.c_alpha, cb = P.c_beta;
    const double kTwoPi = 2.0 * 3.14159265358979311600;
    const double kPi = 3.14159265358979311600;
    const int64_t cap = n;                      // output span = 2n floats (QPSKDeModulator.cs:366)
    uint32_t *bits = (MODE == kModeDemodulate && mine) ? a.bits + s * a.bits_stride_words : nullptr;
    f2 *syms = (SYMS && mine) ? reinterpret_cast<f2 *>(a.syms) + s * a.syms_stride : nullptr;
    uint32_t word = 0;
    int wbits = 0;
    int64_t widx = 0, nbits = 0;
    int64_t nsym = 0;        // symbols emitted by the M&M (capacity check, MuellerMuller.cs:101)
    int64_t ncs = 0;         // symbols through Costas
    bool done = !mine || cnt == 0;
    bool pending = false;    // an M&M symbol waiting for Costas
    float pci = 0.f, pcq = 0.f;
    const f2 *my = ring + lane * kB;
    auto sample = [&](int64_t p) -> f2 {
        return my[((p >> 6) & (kR - 1)) * (SPW * kB) + (p & (kB - 1))];
    };

#ifdef QPSK_LOOP_STAMPS
    unsigned long long c_bar = 0, c_loop = 0, c_iters = 0;
#endif
    for (int r = 0; r < NR; ++r) {
        STAMP(tb);
        __builtin_amdgcn_s_barrier();
        ACC(c_bar, tb);
        STAMP(tl);
        const int64_t rend = (static_cast<int64_t>(r) + 1) * kB < cnt ? (static_cast<int64_t>(r) + 1) * kB : cnt;
        f2 xm1 = sample(base - 1), x0 = sample(base), x1 = sample(base + 1), x2 = sample(base + 2);
        for (;;) {
            const bool can_mm = !done && base + 2 < rend;
            if (!can_mm && !pending) break;

            // ---- Costas + decode on the pending symbol (CostasLoopQpsk.cs:63-92)
            double sn, cs;
            qpsk_sincos(theta, &sn, &cs);
            const double mi = static_cast<double>(pci) * cs + static_cast<double>(pcq) * sn;
            const double mq = static_cast<double>(pcq) * cs - static_cast<double>(pci) * sn;
            const float ri = static_cast<float>(mi), rq = static_cast<float>(mq);
            const float ei = ri >= 0.0f ? 1.0f : -1.0f;
            const float eq = rq >= 0.0f ? 1.0f : -1.0f;
            const double pe = static_cast<double>(ei) * mq - static_cast<double>(eq) * mi;
            const double freq_n = freq + cb * pe;
            double theta_n = theta + (freq_n + ca * pe);
            theta_n = theta_n > kPi ? theta_n - kTwoPi : (theta_n < -kPi ? theta_n + kTwoPi : theta_n);

            // ---- M&M step at (base, mu) (MuellerMuller.cs:62-119), float interp
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
            const double t1 = static_cast<double>(pdi) * ci + static_cast<double>(pdq) * cq;
            const double t2 = static_cast<double>(di) * psi + static_cast<double>(dq) * psq;
            const double e = t1 - t2;
            const double integ_c = integ + ki * e;
            double corr = kp * e + integ_c;
            corr = corr > 0.1 ? 0.1 : corr;
            corr = corr < -0.1 ? -0.1 : corr;
            const double adv = has_prev ? sps + corr : sps;
            const double nt = static_cast<double>(base - d) + mu + adv;
            const double fl = floor(nt);

            // ---- commit Costas / decode
            if (pending) {
                freq = freq_n;
                theta = theta_n;
                if (SYMS) {
                    if (ncs < a.syms_cap) syms[ncs] = f2{ri, rq};
                    else err |= 2;
                }
                ++ncs;
                if (MODE == kModeDemodulate) {
                    // decision + differential decode (QPSKDeModulator.cs:379-407, 304-337)
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
            // ---- commit M&M
            pending = false;
            if (can_mm) {
                integ = has_prev ? integ_c : integ;   // updated even when capacity stops the emit
                has_prev = 1;
                if (nsym >= cap) {
                    done = true;                      // MuellerMuller.cs:101-102
                } else {
                    pending = true;
                    pci = ci;
                    pcq = cq;
                    ++nsym;
                    psi = ci; psq = cq;
                    pdi = di; pdq = dq;
                    base = static_cast<int64_t>(fl) + d;
                    mu = nt - fl;
                    if (base + 1 >= cnt) done = true;
                    // next interpolation taps (stale beyond the round end: then the
                    // loop leaves and they are re-read after the barrier)
                    xm1 = sample(base - 1); x0 = sample(base); x1 = sample(base + 1); x2 = sample(base + 2);
                }
            }
#ifdef QPSK_LOOP_STAMPS
            ++c_iters;
#endif
        }
        ACC(c_loop, tl);
    }
#ifdef QPSK_LOOP_STAMPS
    if (a.probe && lane == 0) {
        a.probe[blockIdx.x * 8 + 3] = c_bar;
        a.probe[blockIdx.x * 8 + 4] = c_loop;
        a.probe[blockIdx.x * 8 + 5] = c_iters;
        a.probe[blockIdx.x * 8 + 6] = NR;
    }
#endif
    if (!mine) return;
    if (cnt == 0) {   // empty DeModulate call: nothing changes
        if (a.n_bits) a.n_bits[s] = 0;
        if (a.n_syms) a.n_syms[s] = 0;
        return;
    }
    if (MODE == kModeDemodulate && wbits > 0) {
        if (widx < a.bits_cap_words) bits[widx] = __builtin_bswap32(word << (32 - wbits));
        else err |= 2;
    }
    // drop consumed samples, keep the rest for the next call (MuellerMuller.cs:123-133)
    const int64_t count = R + n;
    const int64_t lbase = base - d;
    if (a.n_syms) a.n_syms[s] = nsym;
    int64_t consumed = lbase - 1 > 0 ? lbase - 1 : 0;
    const int64_t keep_min = count - 3 > 0 ? count - 3 : 0;
    if (keep_min < consumed) consumed = keep_min;
    int64_t keep = count - consumed;
    if (keep > kCarryMax) {
        err |= 1;
        consumed = count - kCarryMax;
        keep = kCarryMax;
    }
    const f2 *q = reinterpret_cast<const f2 *>(a.mf) + s * a.mf_stride + kMfPrefix - R;  // logical 0
    f2 *cw = reinterpret_cast<f2 *>(a.carry) + static_cast<int64_t>(s) * kCarryMax;
    for (int64_t i = 0; i < keep; ++i) cw[i] = q[consumed + i];
    st.base = static_cast<int32_t>(lbase - consumed);
    st.carry_n = static_cast<int32_t>(keep);
    st.mu = mu;
    st.integ = integ;
    st.psi = psi; st.psq = psq; st.pdi = pdi; st.pdq = pdq;
    st.has_prev = has_prev;
    st.theta = theta;
    st.freq = freq;
    if (MODE == kModeDemodulate) {
        st.diff_have = diff_have;
        st.diff_pi = dpi;
        st.diff_pq = dpq;
    }
    st.error = err;
    a.state[s] = st;
    if (a.n_bits) a.n_bits[s] = MODE == kModeDemodulate ? nbits : 0;
}

template <int SPW>
static void launch_loop_spw(const LoopArgs &a, const LoopParams &P, int mode, hipStream_t stream) {
    dim3 grid((a.S + SPW - 1) / SPW), block(128);
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
    // few streams: spread them over more CUs (the loop is latency-bound per lane)
    if (streams_per_block == 16 || (streams_per_block <= 0 && a.S <= 1024))
        launch_loop_spw<16>(a, P, mode, stream);
    else if (streams_per_block == 32)
        launch_loop_spw<32>(a, P, mode, stream);
    else
        launch_loop_spw<64>(a, P, mode, stream);
}

}  // namespace qpsk
