// qpsk_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the batched QPSK
// demodulation chain.
//
//   fir_tile_kernel    RRC matched filter (ComplexFIRFilter.Filter, FIRFilter.cs:59-91,
//                      144-211) for a [stream][time] batch; LDS-staged input tile
//                      with (T-1)-sample halo, taps as uniform scalar loads, the C# Vector<float>
//                      lane summation order reproduced exactly.
//   fir_generic_kernel same contract for tap counts / lane widths without a
//                      specialised instantiation.
//   fir_hist_kernel    carries the last T-1 input samples to the next call.
//   loop_kernel        MuellerMuller.Process (MuellerMuller.cs:52-190) fused with
//                      CostasLoopQpsk.Process (CostasLoopQpsk.cs:63-92), hard
//                      decision, differential decode and MSB-first bit packing
//                      (QPSKDeModulator.cs:372-408); one lane per stream.
//   fll_kernel         FLLBandEdgeFilter.Process (Band-Edge Filter.cs:64-129),
//                      one lane per stream (any Vector width); the 8-lane
//                      systolic kernel is in qpsk_fll.hip.
//
// Compiled with -ffp-contract=off: every float/double op rounds exactly as the
// reference C# (which never fuses a*b+c).  The only fma() calls are the explicit
// ones inside the portable sincos (qpsk_sincos.h).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "qpsk_kernels.h"
#include "qpsk_sincos.h"

namespace qpsk {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// Matched-filter FIR
// ---------------------------------------------------------------------------
// LDS image of the input tile: one float2 per slot, 8 pad slots after every 64
// samples so the stride-64 groups of a wave's reads fall on distinct banks.
__device__ __forceinline__ int lds_slot(int i) { return i + ((i >> 6) << 3); }
constexpr int lds_slots(int n) { return n + ((n >> 6) << 3) + 8; }

// 2048-output tiles; 1024- and 512-output tiles measured the same
constexpr int kFirThreads = 256;
constexpr unsigned kKtLastWgs = 8192;

// One output of the tile with the reference's full complex products
// (FIRFilter.cs:165-192): lane accumulators from +0, (hI*xI) - (hQ*xQ) and
// (hI*xQ) + (hQ*xI) with hQ = +0 (the RRC's imaginary taps).  The fast path
// drops the hQ products, which is exact for finite samples; a NaN or Inf
// sample makes 0*x NaN, so tiles whose fast outputs are not all finite are
// recomputed here.  x(k) = window sample k (oldest first) from LDS.
// Rolled loops (inlined into the rare branch): few registers, so the fast
// path's allocation is unchanged.
template <typename XF>
__device__ __forceinline__ f2 fir_exact_one(XF x, const float *hrev, int T, int W) {
    const float hq = 0.0f;
    float ai = 0.0f, aq = 0.0f;
    const int nvec = W > 1 ? T - T % W : 0;
#pragma unroll 1
    for (int l = 0; l < (W > 1 ? W : 0); ++l) {
        float vi = 0.0f, vq = 0.0f;
#pragma unroll 1
        for (int k = l; k < nvec; k += W) {
            const f2 u = x(k);
            const float hi = hrev[k];
            vi = vi + ((hi * u.x) - (hq * u.y));
            vq = vq + ((hi * u.y) + (hq * u.x));
        }
        ai += vi;
        aq += vq;
    }
#pragma unroll 1
    for (int k = nvec; k < T; ++k) {
        const f2 u = x(k);
        const float hi = hrev[k];
        ai += (hi * u.x) - (hq * u.y);
        aq += (hi * u.y) + (hq * u.x);
    }
    return f2{ai, aq};
}

// The arithmetic of Q outputs of one thread: row = the thread's LDS row base
// (lds + 72 * grp + r), outputs t0 + W*q, q < Q, t0 = 64*grp + r.  A group of
// W threads covers one 64-sample LDS row of outputs.  The read of input t0 + c
// (c a compile-time offset) lands in slot 72*grp + r + c + 8*floor((r+c)/64);
// the floor is compile-time except when c mod 64 > 56, so almost every ds_read
// uses an immediate offset and the 8-slot row pad keeps the four groups of a
// half-wave on distinct banks.
template <int T, int W, int Q>
__device__ __forceinline__ void fir_core(const f2 *row, int r, const float *hrev, f2 (&acc)[Q]) {
    constexpr int J = T / W;          // full Vector<float> blocks
    constexpr int NVEC = J * W;
    constexpr int TAIL = T - NVEC;    // scalar tail taps (FIRFilter.cs:183-192)
    static_assert(W * Q == 64, "specialised FIR expects W*Q == 64");
    auto rd = [&](int c) -> f2 {
        const int lo = c >> 6, hi = (c + W - 1) >> 6;
        if (lo == hi) return row[c + 8 * lo];
        return row[c + 8 * lo + ((r + (c & 63)) >= 64 ? 8 : 0)];
    };
    // Taps are uniform scalar loads from the device copy, issued per lane phase
    // l behind a compiler barrier, so at most J taps are live at a time (long
    // filters would otherwise spill SGPR taps through v_writelane/v_readlane:
    // +26 % VALU at T = 129).
    typedef __attribute__((address_space(4))) const float cfloat;   // scalar (s_load) path
    cfloat *hc = (cfloat *)hrev;
    auto tap = [&](int idx) -> float { return hc[idx]; };
    if constexpr (J == 0) {
#pragma unroll
        for (int q = 0; q < Q; ++q) acc[q] = f2{0.f, 0.f};
    }
    // Lane accumulator l of every output: sum_j hrev[jW+l] * x[t-T+1+jW+l],
    // j ascending (FIRFilter.cs:165-174); u_i = x[t0 + l + W i] is shared by
    // the Q outputs of this thread.  RD(i) reads u_i.
    auto lane_phase = [&](int l, auto rdu) __attribute__((always_inline)) {
        asm volatile("" ::: "memory");
        f2 A[Q];
#pragma unroll
        for (int i = 0; i < Q + J - 1; ++i) {
            const f2 u = rdu(i);
            f2 p[Q];   // all products of u first, then the adds (no mul->add stall)
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int j = i - q;
                if (j >= 0 && j < J) p[q] = tap(j * W + l) * u;
            }
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int j = i - q;
                if (j >= 0 && j < J) A[q] = (j == 0) ? p[q] : A[q] + p[q];
            }
        }
        // Horizontal sum in lane order 0..W-1 (FIRFilter.cs:176-180).
#pragma unroll
        for (int q = 0; q < Q; ++q) acc[q] = (l == 0) ? A[q] : acc[q] + A[q];
    };
    if constexpr (J > 0 && W == 8) {
        // lane phase 0 unrolled, phases 1..7 as one rolled body: 6.8 KB of code
        // at T = 129 instead of 20.9 KB, and 2 % faster (C3 FIR alone 41.2 ->
        // 40.4 ms, A/B x2, profiles/archive/r02_fir_roll_ab.txt).  With l at run time,
        // input l + 8i sits at row + l + 8i + 8(i/8), plus 8 more when
        // r + l + 8(i%8) >= 64, i.e. i%8 == 7 and r + l >= 8
        lane_phase(0, [&](int i) { return rd(W * i); });
#pragma unroll 1
        for (int l = 1; l < W; ++l) {
            const f2 *rowl = row + l;
            const f2 *rowlw = rowl + ((r + l) >= 8 ? 8 : 0);
            lane_phase(l, [&](int i) {
                const int off = 8 * i + 8 * (i >> 3);
                return (i & 7) == 7 ? rowlw[off] : rowl[off];
            });
        }
    } else {
#pragma unroll
        for (int l = 0; l < W && J > 0; ++l) lane_phase(l, [&](int i) { return rd(l + W * i); });
    }
#pragma unroll
    for (int k = 0; k < TAIL; ++k) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const f2 u = rd(W * q + NVEC + k);
            acc[q] = acc[q] + tap(NVEC + k) * u;
        }
    }
}

__device__ __forceinline__ int fir_nonfinite(float v) { return __builtin_amdgcn_classf(v, 0x207); }   // NaN, +-Inf

// Stage x[tile0-(T-1) .. tile0+TILE) into LDS; t<0 from the previous call's
// history, t>=n as zeros (those outputs are not stored).
template <int T, int NIN, bool VEC, int NT>
__device__ __forceinline__ void fir_stage(f2 *lds, const f2 *x, const f2 *hist, int64_t tile0, int64_t n) {
    const int tid = threadIdx.x;
    const int64_t g0 = tile0 - (T - 1);
    if constexpr (VEC) {
        // g0 is even (T odd) and rows are 16-B aligned: one float4 = 2 samples.
        for (int p = tid; p < (NIN + 1) / 2; p += NT) {
            const int64_t g = g0 + 2 * p;
            f4 v;
            if (g >= 0 && g + 1 < n) {
                v = *reinterpret_cast<const f4 *>(x + g);
            } else {
                f2 lo = g < 0 ? hist[T - 1 + g] : (g < n ? x[g] : f2{0.f, 0.f});
                f2 hi = (g + 1) < 0 ? hist[T + g] : ((g + 1) < n ? x[g + 1] : f2{0.f, 0.f});
                v = f4{lo.x, lo.y, hi.x, hi.y};
            }
            *reinterpret_cast<f4 *>(&lds[lds_slot(2 * p)]) = v;
        }
    } else {
        for (int i = tid; i < NIN; i += NT) {
            const int64_t g = g0 + i;
            lds[lds_slot(i)] = g < 0 ? hist[T - 1 + g] : (g < n ? x[g] : f2{0.f, 0.f});
        }
    }
}

template <int T, int W, int Q, bool VEC, int NT>
__global__ __launch_bounds__(NT) void fir_tile_kernel(FirArgs a, const float *hrev) {
    constexpr int TILE = NT * Q;
    constexpr int NIN = TILE + T - 1;
    __shared__ f2 lds[lds_slots(NIN)];

    const int s = blockIdx.y;
    const int64_t tile0 = static_cast<int64_t>(blockIdx.x) * TILE;
    const int64_t n = a.lengths ? a.lengths[s] : a.n;
    const int tid = threadIdx.x;
    // launch timestamps: workgroups are dispatched in linear order, so the
    // launch starts with the first ones and ends with one of the last
    // kKtLastWgs (a few workgroup lifetimes of the whole chip)
    const unsigned lin = blockIdx.y * gridDim.x + blockIdx.x;
    const bool kt_last = a.kt && tid == 0 && lin + kKtLastWgs >= gridDim.x * gridDim.y;
    if (a.kt && tid == 0 && lin < 64) kt_start(a.kt);
    if (tile0 >= n) {
        if (kt_last) kt_end(a.kt);
        return;
    }
    // shader-clock sample: this workgroup's lifetime in both clocks
    const bool clk_wg = a.clk && tid == 0 && lin % kFirClockEvery == 0;
    unsigned long long c0 = 0, r0 = 0;
    if (clk_wg) {
        c0 = __builtin_amdgcn_s_memtime();
        r0 = wall_clock64();
    }
    const f2 *x = reinterpret_cast<const f2 *>(a.x) + s * a.x_stride;
    const f2 *hist = reinterpret_cast<const f2 *>(a.hist) + static_cast<int64_t>(s) * (T - 1);
    // phase sample: shader-clock stamps at the phase boundaries (the barriers)
    // and whether a loop workgroup holds this CU (glc read: the map entry was
    // written through the XCD's L2 by the loop workgroup on this very CU)
    const bool ph_wg = a.phases && tid == 0 && lin % kFirClockEvery == 0;
    unsigned long long p0 = 0, p1 = 0, p2 = 0;
    unsigned shared_cu = 0;
    if (ph_wg) {
        shared_cu = __hip_atomic_load(a.cu_map + cu_key(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
        p0 = __builtin_amdgcn_s_memtime();
    }

    fir_stage<T, NIN, VEC, NT>(lds, x, hist, tile0, n);
    __syncthreads();
    if (ph_wg) p1 = __builtin_amdgcn_s_memtime();

    const int grp = tid / W, r = tid % W;
    f2 acc[Q];
    fir_core<T, W, Q>(lds + 72 * grp + r, r, hrev, acc);
    // Each output straight from its accumulator: output t0 + W q of lane r of
    // group grp (t0 = 64 grp + r), so a wave's store covers eight 64-B runs.
    // No LDS transpose, no barrier after the compute: the workgroup's LDS is
    // free as soon as its waves are done.  An output whose fast value is not
    // finite had a NaN or Inf in its window and is recomputed with the
    // reference's full products; a finite one had none, and then the fast
    // value is the exact one (fir_exact_one), so the check is per output.
    if (ph_wg) p2 = __builtin_amdgcn_s_memtime();
    {
        f2 *y = reinterpret_cast<f2 *>(a.y) + s * a.y_stride + a.y_offset;
        const int o0 = 64 * grp + r;
        // this thread's outputs from one base address (immediate store
        // offsets); whole tiles, all but a row's last, skip the bounds tests
        f2 *yt = y + tile0 + o0;
        // any non-finite output: 0 * v is +-0 for finite v and NaN for NaN or
        // +-Inf, so z = sum of 0 * acc stays +-0 unless one of them is not
        // finite (an explicit fma: a test, not the reference's arithmetic).
        // One class test instead of one per output (round 6)
        f2 z = f2{0.0f, 0.0f};
#pragma unroll
        for (int q = 0; q < Q; ++q) z = __builtin_elementwise_fma(acc[q], f2{0.0f, 0.0f}, z);
        const bool any_bad = fir_nonfinite(z.x) | fir_nonfinite(z.y);
        if (tile0 + TILE <= n) {
#pragma unroll
            for (int q = 0; q < Q; ++q) yt[W * q] = acc[q];
        } else {
#pragma unroll
            for (int q = 0; q < Q; ++q)
                if (tile0 + o0 + W * q < n) yt[W * q] = acc[q];
        }
        unsigned bad = 0;
        if (__builtin_expect(any_bad, 0)) {
#pragma unroll
            for (int q = 0; q < Q; ++q)
                bad |= static_cast<unsigned>(fir_nonfinite(acc[q].x) | fir_nonfinite(acc[q].y)) << q;
        }
        if (ph_wg) {
            const unsigned long long p3 = __builtin_amdgcn_s_memtime();
            unsigned long long *ph = a.phases + 8 * shared_cu;
            atomicAdd(ph + 0, p1 - p0);
            atomicAdd(ph + 1, p2 - p1);
            atomicAdd(ph + 2, p3 - p2);
            atomicAdd(ph + 3, 1ull);
        }
        if (__builtin_expect(bad != 0, 0)) {
#pragma unroll 1
            for (int q = 0; q < Q; ++q) {
                const int64_t go = tile0 + o0 + W * q;   // output sample
                if (!((bad >> q) & 1u) || go >= n) continue;
                const int64_t w0 = go - (T - 1);         // its oldest window sample
                auto xs = [&](int k) -> f2 {
                    const int64_t g = w0 + k;
                    return g < 0 ? hist[T - 1 + g] : x[g];
                };
                y[go] = fir_exact_one(xs, hrev, T, W);
            }
        }
    }
    if (clk_wg) {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = wall_clock64();
        atomicAdd(a.clk, c1 - c0);
        atomicAdd(a.clk + 1, r1 - r0);
    }
    if (kt_last) kt_end(a.kt);
}

// Any (T, W) without a specialised tile kernel: the reference's formula
// itself, full complex products included (not on the benchmarked path).
__global__ __launch_bounds__(256) void fir_generic_kernel(FirArgs a, const float *hrev, int T,
                                                          int W) {
    const int s = blockIdx.y;
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t n = a.lengths ? a.lengths[s] : a.n;
    const unsigned lin = blockIdx.y * gridDim.x + blockIdx.x;
    if (a.kt && threadIdx.x == 0 && lin < 64) kt_start(a.kt);
    KtEnd kte{lin + kKtLastWgs >= gridDim.x * gridDim.y ? a.kt : nullptr};
    if (t >= n) return;
    const f2 *x = reinterpret_cast<const f2 *>(a.x) + s * a.x_stride;
    const f2 *hist = reinterpret_cast<const f2 *>(a.hist) + static_cast<int64_t>(s) * (T - 1);
    const int64_t w0 = t - T + 1;
    auto xs = [&](int k) -> f2 {
        const int64_t g = w0 + k;
        return g < 0 ? hist[T - 1 + g] : x[g];
    };
    f2 *y = reinterpret_cast<f2 *>(a.y) + s * a.y_stride + a.y_offset;
    y[t] = fir_exact_one(xs, hrev, T, W);
}

// new_hist = last (T-1) samples of concat(old_hist, x[0..n))
__global__ void fir_hist_kernel(FirArgs a, float *hist_new, int H, int S) {
    const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (idx >= static_cast<int64_t>(S) * H) return;
    const int s = static_cast<int>(idx / H);
    const int k = static_cast<int>(idx % H);
    const int64_t n = a.lengths ? a.lengths[s] : a.n;
    const f2 *x = reinterpret_cast<const f2 *>(a.x) + s * a.x_stride;
    const f2 *ho = reinterpret_cast<const f2 *>(a.hist) + static_cast<int64_t>(s) * H;
    f2 *hn = reinterpret_cast<f2 *>(hist_new) + static_cast<int64_t>(s) * H;
    const int64_t m = n + k;
    hn[k] = m < H ? ho[m] : x[m - H];
}

// ---------------------------------------------------------------------------
// Band-Edge FLL, one lane per stream (exact reference order)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void fll_dot(const float *taps_rev, const f2 *win, int W, float *oi,
                                        float *oq) {
    constexpr int N = kFllTaps;
    float acc_i = 0.f, acc_q = 0.f;
    if (W > 1) {
        const int nvec = N - N % W;
        for (int l = 0; l < W; ++l) {
            float vi = 0.f, vq = 0.f;
            for (int i = 0; i < nvec; i += W) {
                const float hi = taps_rev[2 * (i + l)], hq = taps_rev[2 * (i + l) + 1];
                const f2 x = win[i + l];
                vi = vi + ((hi * x.x) - (hq * x.y));
                vq = vq + ((hi * x.y) + (hq * x.x));
            }
            acc_i += vi;
            acc_q += vq;
        }
        for (int i = nvec; i < N; ++i) {
            const float hi = taps_rev[2 * i], hq = taps_rev[2 * i + 1];
            const f2 x = win[i];
            acc_i += (hi * x.x) - (hq * x.y);
            acc_q += (hi * x.y) + (hq * x.x);
        }
    } else {
        for (int i = 0; i < N; ++i) {
            const float hi = taps_rev[2 * i], hq = taps_rev[2 * i + 1];
            const f2 x = win[i];
            acc_i += (hi * x.x) - (hq * x.y);
            acc_q += (hi * x.y) + (hq * x.x);
        }
    }
    *oi = acc_i;
    *oq = acc_q;
}

__global__ __launch_bounds__(64) void fll_kernel(FllArgs a, FllParams P) {
    if (a.kt && threadIdx.x == 0) kt_start(a.kt);
    KtEnd kte{a.kt};
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= a.S) return;
    const int64_t n = a.lengths ? a.lengths[s] : a.n;
    if (n == 0) return;
    constexpr int N = kFllTaps;
    const StreamState *st_in = a.state + s;
    const f2 *x = reinterpret_cast<const f2 *>(a.x) + s * a.x_stride;
    f2 *y = reinterpret_cast<f2 *>(a.y) + s * a.y_stride;
    // 2N delay line (FIRFilter.cs:18-22), shared by both band-edge filters since
    // both are fed the same mixed sample.
    f2 *dl = reinterpret_cast<f2 *>(a.delay) + static_cast<int64_t>(s) * 2 * N;
    float phase = st_in->fll_phase, freq = st_in->fll_freq;
    int pos = st_in->fll_pos;
    const float two_pi = 2.0f * 3.14159274101257324219f;
    for (int64_t t = 0; t < n; ++t) {
        const f2 in = x[t];
        float sn, cs;
        qpsk_sincosf_glibc(phase, &sn, &cs);   // MathF.Cos/Sin = glibc (Band-Edge Filter.cs:108-109)
        const float oi = in.x * cs - in.y * sn;
        const float oq = in.x * sn + in.y * cs;
        y[t] = f2{oi, oq};
        dl[pos] = f2{oi, oq};
        dl[pos + N] = f2{oi, oq};
        int start = pos + 1;
        if (start >= N) start -= N;
        float upi, upq, loi, loq;
        fll_dot(P.upper_rev, dl + start, P.lanes, &upi, &upq);   // filterUpper first (:115)
        fll_dot(P.lower_rev, dl + start, P.lanes, &loi, &loq);
        const float pu = upi * upi + upq * upq;
        const float pl = loi * loi + loq * loq;
        const float err = pl - pu;
        freq += P.beta * err;
        phase += freq + P.alpha * err;
        if (phase > two_pi || phase < -two_pi) phase = remainderf(phase, two_pi);
        if (freq > P.max_freq) freq = P.max_freq;
        else if (freq < P.min_freq) freq = P.min_freq;
        ++pos;
        if (pos == N) pos = 0;
    }
    // only the FLL's own fields: in pipelined calls the loop kernel of the
    // previous call may be writing the M&M/Costas fields of this struct
    a.state[s].fll_phase = phase;
    a.state[s].fll_freq = freq;
    a.state[s].fll_pos = pos;
}

// ---------------------------------------------------------------------------
// IQ_Balancer.Process (IQ Balancer.cs:15-25), the optional pre-stage
// (qpsk_demod_params.iq_balance): per-stream exponential averages of I and Q
// subtracted from the samples, in the reference's float order (mul, then add;
// no fma).  The reference loop stops at IN.Length/2 floats, i.e. half the
// samples; this stage covers every sample ("fixed").  A
// serial recurrence: one lane per stream, two samples per 16-B load.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void iq_balance_kernel(IqbArgs a) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= a.S) return;
    const int64_t n = a.lengths ? a.lengths[s] : a.n;
    if (n <= 0) return;
    const f2 *x = reinterpret_cast<const f2 *>(a.x) + s * a.x_stride;
    f2 *y = reinterpret_cast<f2 *>(a.y) + s * a.y_stride;
    const float ratio = 1e-05f;
    float ar = a.state[s].iqb_re, ai = a.state[s].iqb_im;
    for (int64_t t = 0; t < n; ++t) {
        const f2 v = x[t];
        ar = ratio * (v.x - ar) + ar;
        ai = ratio * (v.y - ai) + ai;
        y[t] = f2{v.x - ar, v.y - ai};
    }
    a.state[s].iqb_re = ar;
    a.state[s].iqb_im = ai;
}

void launch_iq_balance(const IqbArgs &a, hipStream_t stream) {
    hipLaunchKernelGGL(iq_balance_kernel, dim3((a.S + 63) / 64), dim3(64), 0, stream, a);
}

// ---------------------------------------------------------------------------
// Chunked calls: one DeModulate call longer than max_samples_per_call runs as
// consecutive internal chunks (the chain is chunk-invariant), and each chunk's
// bit row / symbol row is appended behind the previous chunk's in the
// caller's row, so the caller sees one call's output (QPSKDeModulator.cs:345-425
// takes any span length).  One workgroup per stream.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void append_rows_kernel(AppendArgs a) {
    const int s = blockIdx.x;
    const int64_t nb = a.counts[s], ns = a.counts[a.S + s];
    const int64_t off = a.first ? 0 : a.acc[s];
    const int64_t offs = a.first ? 0 : a.acc[a.S + s];
    if (a.dst_bits && nb > 0) {
        // dst bit off + i <- src bit i, MSB-first: dst byte base + j takes the
        // low sh bits of src byte j-1 and the high 8-sh bits of src byte j
        const uint8_t *src = reinterpret_cast<const uint8_t *>(a.src_bits + s * a.src_bits_words);
        uint8_t *dst = a.dst_bits + s * a.dst_bits_stride;
        const int sh = static_cast<int>(off & 7);
        const int64_t base = off >> 3;
        const int64_t nsrc = (nb + 7) >> 3;
        const int64_t nout = ((off + nb + 7) >> 3) - base;
        for (int64_t j = threadIdx.x; j < nout; j += blockDim.x) {
            const unsigned cur = j < nsrc ? src[j] : 0u;
            const unsigned prev = j > 0 ? src[j - 1] : 0u;
            unsigned v = ((prev << (8 - sh)) | (cur >> sh)) & 0xffu;
            if (j == 0 && sh) v |= dst[base] & (0xff00u >> sh);   // earlier chunk's bits
            // bits past the end of this chunk are zero in src (the loop kernel
            // pads the last word with zeros); mask them anyway
            if (j == nout - 1) {
                const int tail = static_cast<int>((off + nb) & 7);
                if (tail) v &= 0xff00u >> tail;
            }
            dst[base + j] = static_cast<uint8_t>(v);
        }
    }
    if (a.dst_syms && ns > 0) {
        const float *src = a.src_syms + s * 2 * a.src_syms_cap;
        float *dst = a.dst_syms + s * a.dst_syms_stride + 2 * offs;
        for (int64_t i = threadIdx.x; i < 2 * ns; i += blockDim.x) dst[i] = src[i];
    }
    __syncthreads();   // every thread has read acc
    if (threadIdx.x == 0) {
        a.acc[s] = off + nb;
        a.acc[a.S + s] = offs + ns;
        if (a.last) a.state[s].tofs = 0;   // streams whose samples ended earlier included
    }
}

void launch_append(const AppendArgs &a, hipStream_t stream) {
    hipLaunchKernelGGL(append_rows_kernel, dim3(a.S), dim3(256), 0, stream, a);
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
template <int T, int NT>
static void launch_fir_w8_nt(const FirArgs &a, const float *hrev, int S,
                             int64_t n_max, bool vec, hipStream_t stream) {
    constexpr int Q = 8;
    const int64_t tiles = (n_max + NT * Q - 1) / (NT * Q);
    dim3 grid(static_cast<unsigned>(tiles), static_cast<unsigned>(S));
    if (vec)
        hipLaunchKernelGGL((fir_tile_kernel<T, 8, Q, true, NT>), grid, dim3(NT), 0, stream, a, hrev);
    else
        hipLaunchKernelGGL((fir_tile_kernel<T, 8, Q, false, NT>), grid, dim3(NT), 0, stream, a, hrev);
}

template <int T>
static bool launch_fir_w8(const FirArgs &a, const float *hrev, int S,
                          int64_t n_max, bool vec, hipStream_t stream) {
    // 2048-output tiles; 1024- and 512-output tiles (128 / 64 threads, more
    // workgroups beside the loop kernel's) measured the same at C3 and C2
    // (pipelined bench, A/B x2 on one MI355X), and so did a
    // work-sharing tile whose waves take 512-output units from an LDS counter
    // (profiles/archive/r02_fir_share_ab.txt)
    launch_fir_w8_nt<T, kFirThreads>(a, hrev, S, n_max, vec, stream);
    return true;
}

bool launch_fir(const FirArgs &a, const float *hrev_dev, int T, int W, int S,
                int64_t n_max, hipStream_t stream) {
    if (n_max <= 0 || S <= 0) return true;
    const bool vec = (T % 2 == 1) && ((reinterpret_cast<uintptr_t>(a.x) & 15) == 0) &&
                     (a.x_stride % 2 == 0) && ((reinterpret_cast<uintptr_t>(a.y) & 15) == 0) &&
                     (a.y_stride % 2 == 0) && (a.y_offset % 2 == 0);
    if (W == 8) {
        switch (T) {
        case 13: return launch_fir_w8<13>(a, hrev_dev, S, n_max, vec, stream);
        case 17: return launch_fir_w8<17>(a, hrev_dev, S, n_max, vec, stream);
        case 21: return launch_fir_w8<21>(a, hrev_dev, S, n_max, vec, stream);
        case 33: return launch_fir_w8<33>(a, hrev_dev, S, n_max, vec, stream);
        case 41: return launch_fir_w8<41>(a, hrev_dev, S, n_max, vec, stream);
        case 49: return launch_fir_w8<49>(a, hrev_dev, S, n_max, vec, stream);
        case 65: return launch_fir_w8<65>(a, hrev_dev, S, n_max, vec, stream);
        case 97: return launch_fir_w8<97>(a, hrev_dev, S, n_max, vec, stream);
        case 129: return launch_fir_w8<129>(a, hrev_dev, S, n_max, vec, stream);
        default: break;
        }
    }
    const int threads = 256;
    dim3 grid(static_cast<unsigned>((n_max + threads - 1) / threads), static_cast<unsigned>(S));
    hipLaunchKernelGGL(fir_generic_kernel, grid, dim3(threads), 0, stream, a, hrev_dev, T, W);
    return false;
}

void launch_fir_hist(const FirArgs &a, float *hist_new, int H, int S, hipStream_t stream) {
    if (H <= 0 || S <= 0) return;
    const int64_t total = static_cast<int64_t>(S) * H;
    const int threads = 256;
    hipLaunchKernelGGL(fir_hist_kernel, dim3(static_cast<unsigned>((total + threads - 1) / threads)),
                       dim3(threads), 0, stream, a, hist_new, H, S);
}


void launch_fll(const FllArgs &a, const FllParams &P, hipStream_t stream) {
    // the systolic 8-lane kernel (qpsk_fll.hip) for the reference's Vector<float>
    // width 8, conjugate band-edge taps and alpha = 0 (Band-Edge Filter.cs:55,
    // the only value the reference sets); the one-lane kernel otherwise
    if (P.lanes == 8 && kFllTaps == 40 && P.conj_taps && P.alpha == 0.0f) {
        launch_fll_sys(a, P, stream);
        return;
    }
    const int threads = 64;
    hipLaunchKernelGGL(fll_kernel, dim3((a.S + threads - 1) / threads), dim3(threads), 0, stream, a, P);
}

}  // namespace qpsk
