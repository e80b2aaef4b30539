// qpsk_fll.hip -- Band-Edge FLL (FLLBandEdgeFilter.Process, Band-Edge Filter.cs:
// 102-129, 185-195) as a systolic 8-lane pipeline on gfx950.
//
// The reference band-edge dot product (ComplexDotWindow, FIRFilter.cs:144-211,
// N = 40 taps, Vector<float>.Count = 8) sums, for output o, lane accumulator l
// over window indices i = l + 8j (j = 0..4, window index i holds x[o-39+i]),
// then the 8 accumulators in lane order 0..7.  Lane l's newest input for output
// o is x[o-7+l], so the only work that waits for the newest mixed sample x[m]
// is lane 7's last product for output m, plus the last add of the lane sum.
// Everything else can run earlier, off the per-sample chain:
//
//   8 hardware lanes per stream, lane <-> reference Vector lane l.
//   At step m lane l finishes ITS accumulator for output o = m + 7 - l: the
//   partial sum over x[m-32], x[m-24], x[m-16], x[m-8] (computed during step
//   m-1) plus the product with x[m].  The lane sum S_l(o) = S_{l-1}(o) + acc_l(o)
//   arrives from lane l-1, which finished output o one step earlier: a DPP shift
//   per step.  Lane 7 therefore holds the finished filter output for sample m.
//
//   Lanes of a 16-lane DPP row: two streams interleaved (even / odd lanes), so
//   the shift is row_shr:2 and lane 0 of BOTH streams reads past the row start,
//   which bound_ctrl turns into +0 (the reference's `accI = 0f` start; 0 + a0 ==
//   a0 because a0, itself a sum started at +0, is never -0).
//
//   Lane 7 forms the band powers and the error; the error is broadcast to the
//   stream's 8 lanes (3 DPP moves) and every lane then runs the loop filter,
//   phase wrap, sincos and NCO mix redundantly, so every lane holds x[m+1].
//
//   Upper taps are the conjugates of the lower ones (Band-Edge Filter.cs:
//   176-178), so each complex tap costs 2 packed products shared by both
//   filters: lower = (a xr - b xi, a xi + b xr), upper = (a xr + b xi,
//   a xi - b xr), exactly the reference's (hI*xI) - (hQ*xQ), (hI*xQ) + (hQ*xI)
//   with hQ = -b (x - (-y) == x + y and x + (-y) == x - y in IEEE arithmetic).
//
//   The reference's FLL alpha is the constant 0 (Band-Edge Filter.cs:55), so
//   `phase += freq + alpha * error` (:125) is `phase += freq` here: x + (+-0) == x
//   for every x but +-0; freq just updated by `freq += beta * error` is -0 only
//   if error < 0 (beta > 0; error is never -0), and then alpha * error is -0 too;
//   only error = +-Inf differs (0 * Inf = NaN), and there the reference's NaN
//   phase and this kernel's +-Inf phase, wrapped by IEEERemainder in the same
//   step (:127, :185-189), are both NaN.  launch_fll sends a nonzero alpha to the
//   one-lane kernel.
//
//   Main loop (blocks of 8 samples, 4 per iteration): the 32-sample window of
//   mixed samples the partial sums read lives in registers, four 8-sample groups
//   that rotate with the block position, and a block's outputs overwrite the
//   oldest group in place (sample u of it is dead once step u starts).  The LDS
//   ring serves only the first and the last blocks of a call.  The NCO's
//   sinf/cosf is the lane-split form of qpsk_sincosf.h: the stream's even lanes
//   run glibc's sin polynomial, its odd lanes the cos polynomial, one DPP swap
//   hands each the other's value.
//
// Every float op is the reference's op in the reference's order
// (-ffp-contract=off), so the output equals the one-lane fll_kernel bit for bit.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "qpsk_kernels.h"
#include "qpsk_sincosf.h"

namespace qpsk {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kSysStreams = 32;          // streams per 256-thread block: 8 per wave
constexpr int kRingLen = 64;             // mixed samples per stream: x[t] at t & 63 and (t & 63) + 64
constexpr int kRingRow = 2 * kRingLen + 2;   // +2 entries: a wave's 8 rows hit distinct banks

struct FllSysLds {
    f2 ring[kSysStreams * kRingRow];
    float taps[2 * kFllTaps];            // lower taps, reversed, interleaved (prologue)
};

// {p.x - q.y, p.y + q.x}
__device__ __forceinline__ f2 add_swap_neglo(f2 p, f2 q) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(p), "v"(q));
    return r;
}
// {p.x + q.y, p.x - q.y}
__device__ __forceinline__ f2 add_xy_neghi(f2 p, f2 q) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(p), "v"(q));
    return r;
}
// {p.y - q.x, p.y + q.x}
__device__ __forceinline__ f2 add_yx_neglo(f2 p, f2 q) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(p), "v"(q));
    return r;
}

template <int CTRL, int ROWM, int BANKM, bool BC>
__device__ __forceinline__ float dpp(float old, float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old),
                                                                 __builtin_bit_cast(int, v), CTRL, ROWM,
                                                                 BANKM, BC));
}
// lane i <- lane i-2 of its 16-lane row; row lanes 0, 1 (reference lane 0 of
// both streams) read +0
__device__ __forceinline__ float shr2(float v) { return dpp<0x112, 0xf, 0xf, true>(0.0f, v); }
// every lane <- reference lane 7 of its stream: row lane 14 (even lanes'
// stream) or 15 (odd lanes'), row_newbcast:14 / :15 and a select on the lane's
// parity (two independent DPP reads of v instead of a chain of three)
__device__ __forceinline__ float bcast7(float v, bool odd) {
    const int vi = __float_as_int(v);
    const float e14 = __int_as_float(__builtin_amdgcn_mov_dpp(vi, 0x15E, 0xf, 0xf, false));
    const float e15 = __int_as_float(__builtin_amdgcn_mov_dpp(vi, 0x15F, 0xf, 0xf, false));
    return odd ? e15 : e14;
}

// sinf / cosf of y (|y| < 120 or NaN) by the lane-split form (qpsk_sincosf.h):
// this lane's polynomial, its sign, a swap with the partner lane (l ^ 1 = row
// lane +-2: quad_perm [2,3,0,1]) and the pick.  y must not be -0 unless ZFIX,
// which keeps sin(-0) = -0 on the sin lanes (zy = 0 there, NaN on cos lanes).
template <bool ZFIX>
__device__ __forceinline__ void sincosf_split(float y, const qpsk_sincosf_lane &K, uint32_t signv, float zy,
                                              float &sn, float &cs) {
    uint32_t own, t;
#define QPSK_FLL_SELECT(x, x2) (K.sin_lane ? (x) : (x2))
    QPSK_SINCOSF_SPLIT_OWN(y, K, signv, QPSK_FLL_SELECT, own, t);
#undef QPSK_FLL_SELECT
    if constexpr (ZFIX) own = y == zy ? __float_as_uint(y) : own;
    const uint32_t other = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(own), 0x4E, 0xf, 0xf, false));
    uint32_t so, co, m;
    asm("v_bfe_i32 %2, %3, 30, 1\n\tv_bfi_b32 %0, %2, %4, %5\n\tv_bfi_b32 %1, %2, %5, %4"
        : "=&v"(so), "=&v"(co), "=&v"(m)
        : "v"(t), "v"(own), "v"(other));
    sn = __uint_as_float(so);
    cs = __uint_as_float(co);
}

// Band-edge products of complex tap (a, b) [packed A = {a, a}, B = {b, b}] with
// sample x, in the layout the lane sum and the powers want:
//   R = {upper re, lower re} = {a xr + b xi, a xr - b xi}
//   I = {upper im, lower im} = {a xi - b xr, a xi + b xr}
__device__ __forceinline__ void band_prod(f2 A, f2 B, f2 x, f2 &R, f2 &I) {
    const f2 p = A * x;   // {a xr, a xi}
    const f2 q = B * x;   // {b xr, b xi}
    R = add_xy_neghi(p, q);
    I = add_yx_neglo(p, q);
}
// the same with the tap as one register pair T = {a, b}: the broadcasts are
// op_sel / op_sel_hi modifiers of the two v_pk_mul_f32 (half the tap VGPRs)
__device__ __forceinline__ void band_prod(f2 T, f2 x, f2 &R, f2 &I) {
    const f2 p = T.xx * x;   // {a xr, a xi}
    const f2 q = T.yy * x;   // {b xr, b xi}
    R = add_xy_neghi(p, q);
    I = add_yx_neglo(p, q);
}
// The same products with the sign-split sums as one v_pk_fma_f32 each: q times
// +-1 is exact, so fma(q, +-1, p) rounds p +- q once, as the reference's add or
// subtraction (signed zeros, infinities and NaN alike); the compiler folds the
// half-swizzles into op_sel.  Used for the partial sums, off the per-sample
// chain: there they replace inline asm, which hipcc pads with an s_nop at each
// boundary next to a dependent op and between consecutive statements (602 ->
// 580 instructions per block with the scalar redo test, C5 FLL cycles per
// sample -1.2 %, profiles/r05_fll_pkfma_ab.txt).  On the chain the asm form
// measured faster.  KP = {1, -1}, KN = {-1, 1}, pinned in VGPRs by the caller.
__device__ __forceinline__ void band_prod_fma(f2 T, f2 x, f2 KP, f2 KN, f2 &R, f2 &I) {
    const f2 p = T.xx * x;   // {a xr, a xi}
    const f2 q = T.yy * x;   // {b xr, b xi}
    R = __builtin_elementwise_fma(q.yy, KP, p.xx);   // {p.x + q.y, p.x - q.y}
    I = __builtin_elementwise_fma(q.xx, KN, p.yy);   // {p.y - q.x, p.y + q.x}
}

// one wave per SIMD (C5: 1024 waves on 1024 SIMDs): the whole VGPR file is
// this wave's, so the scheduler need not keep 256 free for a second one
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void fll_sys_kernel(FllArgs a, FllParams P) {
    constexpr int N = kFllTaps;
    static_assert(N == 40, "systolic FLL assumes 5 blocks of 8 taps");
    __shared__ FllSysLds L;
    if (a.kt && threadIdx.x == 0) kt_start(a.kt);
    ClkSample clk{threadIdx.x == 0 ? a.clk : nullptr};
    if (threadIdx.x < 2 * N) L.taps[threadIdx.x] = P.lower_rev[threadIdx.x];

    const int lane = threadIdx.x & 63;
    const int rl = lane & 15;
    const int g = (threadIdx.x >> 4) * 2 + (rl & 1);   // stream within the block
    const int l = rl >> 1;                               // reference Vector lane
    const int s = blockIdx.x * kSysStreams + g;
    const bool valid = s < a.S;
    const int sv = valid ? s : 0;
    const int64_t n = valid ? (a.lengths ? a.lengths[s] : a.n) : 0;
    // the row's LDS address lives in one VGPR (opaque), so every ring access is
    // that register plus a small immediate: pairs merge into ds_read2/ds_write2
    typedef __attribute__((address_space(3))) f2 lds_f2;
    uint32_t ring_addr = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_f2 *)(L.ring + g * kRingRow)));
    asm volatile("" : "+v"(ring_addr));
    // rows are 1040 B apart from a 16-B aligned base: telling the compiler lets it
    // pair the ring accesses into ds_read2_b64 / ds_write2_b64 (the opaque base
    // alone hides the alignment)
    lds_f2 *ring = reinterpret_cast<lds_f2 *>(
        __builtin_assume_aligned(reinterpret_cast<lds_f2 *>(static_cast<uintptr_t>(ring_addr)), 16));
    const f2 *x = reinterpret_cast<const f2 *>(a.x) + sv * a.x_stride;
    f2 *y = reinterpret_cast<f2 *>(a.y) + sv * a.y_stride;

    StreamState *stp = a.state + sv;
    float phase = valid ? stp->fll_phase : 0.f, freq = valid ? stp->fll_freq : 0.f;
    const int pos0 = valid ? stp->fll_pos : 0;

    // ring <- x[-39..-1] from the reference's 2N delay line: the sample written
    // k calls to Filter ago sits at (pos - k) mod N (FIRFilter.cs:61-75)
    const f2 *dly = reinterpret_cast<const f2 *>(a.delay) + static_cast<int64_t>(sv) * 2 * N;
    for (int k = 1 + l; k < N; k += 8) {
        int q = pos0 - k;
        q += q < 0 ? N : 0;
        const f2 v = valid ? dly[q] : f2{0.f, 0.f};
        const int idx = (-k) & (kRingLen - 1);
        ring[idx] = v;
        ring[idx + kRingLen] = v;
    }
    __syncthreads();

    // taps of this lane: reversed index l + 8j, as {a, a} and {b, b} pairs
    f2 TA[5], TB[5], TT[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const float ta = L.taps[2 * (l + 8 * j)], tb = L.taps[2 * (l + 8 * j) + 1];
        TA[j] = f2{ta, ta};
        TB[j] = f2{tb, tb};
        TT[j] = f2{ta, tb};
    }

    // pipeline state as after step -1: lane l (< 7) holds the lane sum over
    // lanes 0..l for output 6 - l (reference order: +0, then lanes in order)
    f2 SR = f2{0.f, 0.f}, SI = f2{0.f, 0.f};
    if (l < 7) {
        for (int k = 0; k <= l; ++k) {
            f2 ar = f2{0.f, 0.f}, ai = f2{0.f, 0.f};
            for (int j = 0; j < 5; ++j) {
                const float ta = L.taps[2 * (k + 8 * j)], tb = L.taps[2 * (k + 8 * j) + 1];
                f2 R, I;
                band_prod(f2{ta, ta}, f2{tb, tb}, ring[(-33 + 8 * j + k - l) & (kRingLen - 1)], R, I);
                ar = ar + R;
                ai = ai + I;
            }
            SR = SR + ar;
            SI = SI + ai;
        }
    }
    // partial accumulators of the step at time t (inputs x[t-32], x[t-24],
    // x[t-16], x[t-8]); fetch(k) = x[(t - off) - 32 + k], off <= 8: from the ring
    // (rb = ring + ((t - off - 32) & 63), static offsets, the mirror covers the
    // wrap) or from a block's register window
    f2 PR, PI;
    auto partial = [&](auto fetch, int off) __attribute__((always_inline)) {
        // the reference starts each lane accumulator at +0 (Vector<float>.Zero);
        // 0 + v differs from v only in the sign of a zero, and the filter
        // outputs are only ever squared (the band powers), so the start is dropped
        f2 ar, ai;
        band_prod(TA[0], TB[0], fetch(off), ar, ai);
#pragma unroll
        for (int j = 1; j < 4; ++j) {
            f2 R, I;
            band_prod(TA[j], TB[j], fetch(off + 8 * j), R, I);
            ar = ar + R;
            ai = ai + I;
        }
        PR = ar;
        PI = ai;
    };
    auto ring_at = [&](int64_t t0) __attribute__((always_inline)) {
        const lds_f2 *rb = ring + ((t0 - 32) & (kRingLen - 1));
        return [rb](int k) -> f2 { return rb[k]; };
    };
    partial(ring_at(0), 0);

    const float two_pi = 2.0f * 3.14159274101257324219f;
    // the partial sums' sign vectors, pinned (as SGPR pairs the compiler
    // rebuilt one from the other with two s_mov every block)
    f2 KP = f2{1.0f, -1.0f}, KN = f2{-1.0f, 1.0f};
    asm volatile("" : "+v"(KP), "+v"(KN));
    // the float sign bit in a VGPR for the sincos quadrant logic (v_bitop3_b32
    // takes no literal): pinned once here, not rebuilt every sample
    uint32_t sign_v = 0x80000000u;
    asm volatile("" : "+v"(sign_v));
    const float beta = P.beta, fmax_ = P.max_freq, fmin_ = P.min_freq;
    const bool odd = rl & 1;   // which stream of the DPP row (bcast7)
    // lane-split sincos: even reference lanes evaluate the sin polynomial
    const qpsk_sincosf_lane K = qpsk_sincosf_lane_init((l & 1) == 0);
    const float zy = (l & 1) == 0 ? 0.0f : __builtin_nanf("");

    // one sample (Band-Edge Filter.cs:102-129) at t = t0 + u, t0 a multiple of 8.
    // FIRST: the call's first sample (the stored phase may be anything set_state
    // put there).  EXACT: the IEEERemainder wrap (:185-189) behind a vote and the
    // frequency clamp (:191-195).  Without EXACT the step tracks max |phase| and
    // max |freq| instead, and the block is redone exactly if either left its
    // range (the phase every ~2pi/|freq| samples, the clamp essentially never),
    // so a block is branch-free straight-line code.
    // REG: a uniform block's step -- the partial sums read the block's register
    // window X (x[t0-32 .. t0-1]; x[t0] is this block's first output, xmv[0])
    // and the outputs stay in xmv until the block writes them to the ring at its
    // end (16-B LDS accesses instead of a read per tap and a write pair per
    // sample); otherwise the ring is read and written per sample
    auto step = [&](f2 in, int64_t t0, int u, auto first, auto exact, float &amax, float &fmx,
                    auto reg, const f2 *X, f2 *xmv) __attribute__((always_inline)) {
        // MathF.Cos / MathF.Sin (Band-Edge Filter.cs:108-109) = glibc cosf / sinf
        float sn, cs;
        if constexpr (decltype(first)::value) {
            qpsk_sincosf_glibc(phase, &sn, &cs);
        } else {
            // a kept result has |phase| <= 2pi (or NaN): the branch-free form
            qpsk_sincosf_glibc_fast_k(phase, &sn, &cs, sign_v);
        }
        // (inI*c - inQ*s, inI*s + inQ*c) from p = in*c = {inI*c, inQ*c} and
        // q = in*s = {inI*s, inQ*s}: {p.x - q.y, p.y + q.x}.  The broadcasts are
        // op_sel_hi modifiers of one v_pk_mul_f32 each (plain vector code: no
        // inline asm, whose hazards the compiler pads with s_nop)
        const f2 xm = add_swap_neglo(in * f2{cs, cs}, in * f2{sn, sn});
        if constexpr (decltype(reg)::value) {
            xmv[u] = xm;
        } else {
            lds_f2 *wb = ring + (t0 & (kRingLen - 1));
            wb[u] = xm;
            wb[u + kRingLen] = xm;
        }
        y[t0 + u] = xm;
        f2 R4, I4;
        band_prod(TA[4], TB[4], xm, R4, I4);
        const f2 ar = PR + R4, ai = PI + I4;
        SR = f2{shr2(SR.x) + ar.x, shr2(SR.y) + ar.y};
        SI = f2{shr2(SI.x) + ai.x, shr2(SI.y) + ai.y};
        // lane 7 holds the filter outputs of sample t: {pow upper, pow lower}
        const f2 pw = SR * SR + SI * SI;
        const float err = bcast7(pw.y - pw.x, odd);
        freq = freq + beta * err;
        phase = phase + freq;   // alpha == 0 (file comment)
        if constexpr (decltype(exact)::value) {
            if (__builtin_expect(__ballot(fabsf(phase) > two_pi) != 0, 0))
                if (fabsf(phase) > two_pi) phase = remainderf(phase, two_pi);
            freq = freq > fmax_ ? fmax_ : (freq < fmin_ ? fmin_ : freq);
        } else {
            amax = fmaxf(amax, fabsf(phase));   // NaN never wraps or clamps: ignored
            fmx = fmaxf(fmx, fabsf(freq));
        }
        if constexpr (decltype(reg)::value)
            partial([&](int k) -> f2 { return k == 32 ? xmv[0] : X[k]; }, u + 1);
        else
            partial(ring_at(t0), u + 1);
    };
    // 8 samples of every stream of the wave, no masks
    typedef __attribute__((address_space(3))) f4 lds_f4;
    auto block = [&](const f2 *in, int64_t t0, auto first) __attribute__((always_inline)) {
        const float ph0 = phase, fr0 = freq;
        const f2 sr0 = SR, si0 = SI, pr0 = PR, pi0 = PI;
        float amax = 0.f, fmx = 0.f;
        // the window x[t0-32 .. t0-1]: (t0 - 32) & 63 is a multiple of 8 samples,
        // so 16 aligned 16-B reads (the mirror keeps it contiguous)
        f2 X[32], xmv[8];
        const lds_f4 *wr = reinterpret_cast<const lds_f4 *>(ring + ((t0 - 32) & (kRingLen - 1)));
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const f4 v = wr[k];
            X[2 * k] = f2{v.x, v.y};
            X[2 * k + 1] = f2{v.z, v.w};
        }
        step(in[0], t0, 0, first, std::false_type{}, amax, fmx, std::true_type{}, X, xmv);
#pragma unroll
        for (int u = 1; u < 8; ++u)
            step(in[u], t0, u, std::false_type{}, std::false_type{}, amax, fmx, std::true_type{}, X, xmv);
        if (__builtin_expect(__ballot((amax > two_pi) | (fmx > fmax_)) != 0, 0)) {
            // some stream's phase needed a wrap or its frequency a clamp: redo
            // from the block start (its outputs are rewritten)
            phase = ph0; freq = fr0; SR = sr0; SI = si0; PR = pr0; PI = pi0;
            step(in[0], t0, 0, first, std::true_type{}, amax, fmx, std::true_type{}, X, xmv);
#pragma unroll
            for (int u = 1; u < 8; ++u)
                step(in[u], t0, u, std::false_type{}, std::true_type{}, amax, fmx, std::true_type{}, X, xmv);
        }
        // the block's outputs into the ring and its mirror: x[t0 .. t0+7] at
        // t0 & 63, a multiple of 8 samples (64-B aligned)
        lds_f4 *ww = reinterpret_cast<lds_f4 *>(ring + (t0 & (kRingLen - 1)));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const f4 v = f4{xmv[2 * k].x, xmv[2 * k].y, xmv[2 * k + 1].x, xmv[2 * k + 1].y};
            ww[k] = v;
            ww[k + kRingLen / 2] = v;
        }
    };

    // wave-uniform block counts (8 streams per wave); rows past the batch count
    // as empty streams, so only full waves take the unmasked path
    int64_t nmax = n, nmin = n;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t w1 = __shfl_xor(nmax, o, 64), w2 = __shfl_xor(nmin, o, 64);
        nmax = w1 > nmax ? w1 : nmax;
        nmin = w2 < nmin ? w2 : nmin;
    }
    // Input: every lane of a stream loads the stream's 8 samples of a block
    // (the same addresses for its 8 lanes).  Blocks run from two register
    // buffers A and B, each reloaded right after its block, so a buffer's loads
    // have a whole block to land.
    auto load8 = [&](f2 *buf, int64_t t0) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < 8; ++u) buf[u] = x[t0 + u];
    };

    // ---- register-window blocks ------------------------------------------
    // G[(p + i) & 3] holds x[t0 - 32 + 8i .. t0 - 25 + 8i] at block position p;
    // step u overwrites G[p][u] with the block's output x[t0 + u].  The partial
    // sums of steps 1..7 depend on the old window only (their newest input is
    // x[t0 + u - 7]), so they are kept for a redo; step 8's (the next block's
    // step 0) reads x[t0] = G[p][0], the block's first output.
    f2 G[4][8];
    // lanes whose block-start phase is -0 (sincosf_split<false> excludes it),
    // as a ballot mask: the per-block redo test below is then two compares
    // into SGPR masks, scalar ors and one branch on SCC
    uint64_t need_exact = 0;
    auto rblock = [&](auto pc, const f2 *in, int64_t t0) __attribute__((always_inline)) {
        constexpr int p = decltype(pc)::value;
        auto X = [&](int k) __attribute__((always_inline)) -> f2 { return G[(p + (k >> 3)) & 3][k & 7]; };
        const float ph0 = phase, fr0 = freq;
        const f2 sr0 = SR, si0 = SI;
        f2 QR[9], QI[9];
        QR[0] = PR;
        QI[0] = PI;
        auto part = [&](int u) __attribute__((always_inline)) {   // QR/QI[u + 1]
            f2 ar, ai;
            band_prod_fma(TT[0], X(u + 1), KP, KN, ar, ai);
#pragma unroll
            for (int j = 1; j < 4; ++j) {
                f2 R, I;
                band_prod_fma(TT[j], X(u + 1 + 8 * j), KP, KN, R, I);
                ar = ar + R;
                ai = ai + I;
            }
            QR[u + 1] = ar;
            QI[u + 1] = ai;
        };
        float amax = 0.f, fmx = 0.f;
        auto core = [&](f2 inu, int u, auto exact) __attribute__((always_inline)) {
            float sn, cs;
            sincosf_split<decltype(exact)::value>(phase, K, sign_v, zy, sn, cs);
            const f2 xm = add_swap_neglo(inu * f2{cs, cs}, inu * f2{sn, sn});
            G[p][u] = xm;
            f2 R4, I4;
            band_prod(TT[4], xm, R4, I4);
            const f2 ar = QR[u] + R4, ai = QI[u] + I4;
            SR = f2{shr2(SR.x) + ar.x, shr2(SR.y) + ar.y};
            SI = f2{shr2(SI.x) + ai.x, shr2(SI.y) + ai.y};
            const f2 pw = SR * SR + SI * SI;
            const float err = bcast7(pw.y - pw.x, odd);
            freq = freq + beta * err;
            phase = phase + freq;   // alpha == 0 (file comment)
            if constexpr (decltype(exact)::value) {
                if (__builtin_expect(__ballot(fabsf(phase) > two_pi) != 0, 0))
                    if (fabsf(phase) > two_pi) phase = remainderf(phase, two_pi);
                freq = freq > fmax_ ? fmax_ : (freq < fmin_ ? fmin_ : freq);
            } else {
                amax = fmaxf(amax, fabsf(phase));   // NaN never wraps or clamps: ignored
                fmx = fmaxf(fmx, fabsf(freq));
            }
        };
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            core(in[u], u, std::false_type{});
            part(u);
        }
        const uint64_t redo = __builtin_amdgcn_ballot_w64(amax > two_pi) | __builtin_amdgcn_ballot_w64(fmx > fmax_);
        if (__builtin_expect((redo | need_exact) != 0, 0)) {
            // a wrap, a clamp or a -0 phase: redo the block exactly from its start
            phase = ph0; freq = fr0; SR = sr0; SI = si0;
#pragma unroll
            for (int u = 0; u < 8; ++u) core(in[u], u, std::true_type{});
            part(7);
            // IEEERemainder can return -0 (an exact multiple of 2pi); a fast
            // block never creates -0 (x + y == -0 needs x == -0)
            need_exact = __builtin_amdgcn_ballot_w64(__float_as_uint(phase) == 0x80000000u);
        }
        PR = QR[8];
        PI = QI[8];
    };
    // the block's outputs, stored after the next input loads are issued: a
    // wait for a load (vmcnt counts loads and stores in issue order) then never
    // waits for the stores of the block before it.  With the drain before the
    // loop: C5 FLL 161.3 -> 157.2 ms, 361.4 -> 347.8 cycles per sample (A/B x2
    // on one MI355X, profiles/r05_fll_store_late_ab.txt)
    auto store8 = [&](auto pc, int64_t t0) __attribute__((always_inline)) {
        constexpr int p = decltype(pc)::value;
#pragma unroll
        for (int u = 0; u < 8; ++u) y[t0 + u] = G[p][u];
    };

    int64_t t0 = 0;
    if (nmin >= 56) {
        {   // the call's first block (the full sinf/cosf on its first sample) from the ring
            f2 cur[8];
            load8(cur, 0);
            block(cur, 0, std::true_type{});
        }
        t0 = 8;
        // window x[t0-32 .. t0-1] from the ring: 16 aligned 16-B reads
        const lds_f4 *wr = reinterpret_cast<const lds_f4 *>(ring + ((t0 - 32) & (kRingLen - 1)));
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const f4 v = wr[k];
            G[k >> 2][(2 * k) & 7] = f2{v.x, v.y};
            G[k >> 2][(2 * k + 1) & 7] = f2{v.z, v.w};
        }
        need_exact = __builtin_amdgcn_ballot_w64(__float_as_uint(phase) == 0x80000000u);
        f2 A[8], B[8];
        load8(A, t0);
        load8(B, t0 + 8);
        // drain once per call: the loop is then entered with nothing in flight,
        // and the compiler's vmcnt model of the loop body is the steady state's
        // (from the preheader it would assume A's loads were followed by B's
        // only, and wait for nearly every load of the first blocks)
        // 0xF70 = vmcnt(0) with expcnt / lgkmcnt not waited under the gfx9
        // s_waitcnt field layout only; another target's layout would wait on
        // the wrong counters without a word from the compiler
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "qpsk_fll.hip: the raw s_waitcnt immediate assumes gfx950 (gfx9 field layout)"
#endif
        __builtin_amdgcn_s_waitcnt(0xF70);
        do {
            rblock(std::integral_constant<int, 0>{}, A, t0);
            load8(A, t0 + 16);
            store8(std::integral_constant<int, 0>{}, t0);
            rblock(std::integral_constant<int, 1>{}, B, t0 + 8);
            load8(B, t0 + 24);
            store8(std::integral_constant<int, 1>{}, t0 + 8);
            rblock(std::integral_constant<int, 2>{}, A, t0 + 16);
            load8(A, t0 + 32);
            store8(std::integral_constant<int, 2>{}, t0 + 16);
            rblock(std::integral_constant<int, 3>{}, B, t0 + 24);
            load8(B, t0 + 40);
            store8(std::integral_constant<int, 3>{}, t0 + 24);
            t0 += 32;
        } while (t0 + 48 <= nmin);
        // the window back into the ring (and its mirror) for the blocks that
        // follow: group i at (t0 - 32 + 8i) & 63, a multiple of 8 samples
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            lds_f4 *ww = reinterpret_cast<lds_f4 *>(ring + ((t0 - 32 + 8 * i) & (kRingLen - 1)));
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const f4 v = f4{G[i][2 * k].x, G[i][2 * k].y, G[i][2 * k + 1].x, G[i][2 * k + 1].y};
                ww[k] = v;
                ww[k + kRingLen / 2] = v;
            }
        }
    }
    // the rest (ragged streams, short calls, partly filled waves), block by block
    for (; t0 < nmax; t0 += 8) {
        f2 cur[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) cur[u] = t0 + u < n ? x[t0 + u] : f2{0.f, 0.f};
        if (t0 + 8 <= nmin) {
            if (t0 == 0) block(cur, t0, std::true_type{});
            else block(cur, t0, std::false_type{});
        } else {
            float amax = 0.f, fmx = 0.f;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (t0 + u < n) {
                    if (t0 + u == 0)
                        step(cur[u], t0, u, std::true_type{}, std::true_type{}, amax, fmx, std::false_type{},
                             nullptr, nullptr);
                    else
                        step(cur[u], t0, u, std::false_type{}, std::true_type{}, amax, fmx, std::false_type{},
                             nullptr, nullptr);
                }
        }
    }

    if (n > 0) {
        // the 2N delay line as the reference leaves it: position q holds the
        // newest sample written there, x[n-1 - ((pos_end - 1 - q) mod N)]
        const int pos_end = static_cast<int>((pos0 + n) % N);
        f2 *dw = reinterpret_cast<f2 *>(a.delay) + static_cast<int64_t>(s) * 2 * N;
        for (int q = l; q < N; q += 8) {
            int back = pos_end - 1 - q;
            back += back < 0 ? N : 0;
            const f2 v = ring[(n - 1 - back) & (kRingLen - 1)];
            dw[q] = v;
            dw[q + N] = v;
        }
        if (l == 0) {
            stp->fll_phase = phase;
            stp->fll_freq = freq;
            stp->fll_pos = pos_end;
        }
    }
    if (a.kt && lane == 0) kt_end(a.kt);
}

void launch_fll_sys(const FllArgs &a, const FllParams &P, hipStream_t stream) {
    hipLaunchKernelGGL(fll_sys_kernel, dim3((a.S + kSysStreams - 1) / kSysStreams), dim3(256), 0, stream, a,
                       P);
}

}  // namespace qpsk
