// tools/variants/qpsk_fll_pair.hip -- MEASURED AND REJECTED A/B variant of
// csrc/qpsk_fll.hip (not built by the Makefile; tools/ab_build_fll.sh NAME
// tools/variants/qpsk_fll_pair.hip builds it into _build/ab/libNAME.so).
// A chain wave and a helper wave per SIMD: the helper computes three of the
// four partial band-edge products one block ahead and hands them over through
// LDS; the chain wave runs the NCO with both glibc polynomials side by side and
// a shifter-fma quadrant (checked, redo on a near-tie).  Bit-exact (GPU suite
// FLL/C5 cases green) but slower at C5: 429 cycles/sample with per-pair LDS
// flags, 485 with s_barrier hand-over, against 393 for the product kernel
// (profiles/r04_fll_variants_ab.txt).
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

// the shifter-quadrant sinf/cosf this variant's chain wave used (exact where
// |y * 2/pi - n| <= QPSK_SINCOSF_UMAX, checked on all 2^32 inputs in round 4)
#define QPSK_SINCOSF_UMAX (0.5 - 0x1p-22)
__device__ static inline double qpsk_sincosf_shifter_k(float y, float *s, float *c, uint32_t SIGNV)
{
    const double yd = (double)y;
    const double t = fma(yd, 0x1.45F306DC9C883p-1, 0x1.8p52);
    const double nd = t - 0x1.8p52;
    const double u = fma(yd, 0x1.45F306DC9C883p-1, -nd);
    const int n = (int)(uint32_t)__double_as_longlong(t);
    const double x = fma(-nd, 0x1.921FB54442D18p0, yd);
    const double x2 = x * x;
    const uint32_t t1 = (uint32_t)n << 30;
    uint64_t xb = (uint64_t)__double_as_longlong(x);
    const uint32_t xhi = (uint32_t)(xb >> 32) ^ ((t1 + 0x40000000u) & SIGNV);
    xb = ((uint64_t)xhi << 32) | (uint32_t)xb;
    const double xs = __longlong_as_double((long long)xb);
    const double x3 = xs * x2;
    const double s1 = fma(x2, -0x1.994eb3774cf24p-13, 0x1.1107605230bc4p-7);
    const double x7 = x3 * x2;
    const double sp = fma(x7, s1, fma(x3, -0x1.555545995a603p-3, xs));
    const double x4 = x2 * x2;
    const double c2 = fma(x2, 0x1.99343027bf8c3p-16, -0x1.6c087e89a359dp-10);
    const double c1 = fma(x2, -0x1.ffffffd0c621cp-2, 0x1p0);
    const double x6 = x4 * x2;
    const double cp = fma(x6, c2, fma(x4, 0x1.55553e1068f19p-5, c1));
    const uint32_t fcb = __float_as_uint((float)cp) ^ (t1 & SIGNV);
    const uint32_t fsb = __float_as_uint((float)sp);
    uint32_t so, co, odd;
    asm("v_bfe_i32 %2, %3, 0, 1\n\tv_bfi_b32 %0, %2, %4, %5\n\tv_bfi_b32 %1, %2, %5, %4"
        : "=&v"(so), "=&v"(co), "=&v"(odd)
        : "v"(n), "v"(fcb), "v"(fsb));
    *s = __uint_as_float(so);
    *c = __uint_as_float(co);
    return fabs(u);
}

#ifndef QPSK_FLL_PROBE
#define QPSK_FLL_PROBE 0   // diagnostic bits (timing only, results wrong): 1 no sincos, 2 no
                           // partial sums, 4 no broadcast, 8 no redo, 16 helper idle (no
                           // partial sums), 32 no pair barriers; 0 = product
#endif

namespace qpsk {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kSysStreams = 32;          // streams per block: 8 per chain wave
constexpr int kSysChain = 256;           // chain threads: 4 waves x 8 streams x 8 lanes
constexpr int kSysThreads = 2 * kSysChain;   // + 4 helper waves (one per chain wave)
constexpr int kRingLen = 64;             // mixed samples per stream: x[t] at t & 63 and (t & 63) + 64
constexpr int kRingRow = 2 * kRingLen + 2;   // +2 entries: a wave's 8 rows hit distinct banks
constexpr int kMinPairBlocks = 4;        // shorter calls run on the chain waves alone

struct FllSysLds {
    f2 ring[kSysStreams * kRingRow];
    // helper -> chain: the 3-term partial sums {R, I} of every chain thread for
    // the 8 steps of a block, double-buffered by block parity
    f4 part[2][8][kSysChain];
    float taps[2 * kFllTaps];            // lower taps, reversed, interleaved (prologue)
    unsigned long long nmin;             // the block's shortest stream (uniform pair-loop count)
    // per chain wave w: blocks the chain wave has written to the ring, and
    // blocks of partial sums its helper wave has written (the pair's hand-over)
    int chain_done[4], helper_done[4];
};

// The chain / helper hand-over: a wave publishes a count in LDS after the data
// it covers (LDS serves a wave's accesses in order), and the other wave of the
// pair waits until the count reaches what it needs.  Only the two waves of a
// pair wait for each other (an s_barrier would hold all eight waves to the
// slowest chain wave, e.g. one redoing a block); no wait on global memory.
__device__ __forceinline__ void pair_publish(int *flag, int v) {
    __atomic_store_n(flag, v, __ATOMIC_RELAXED);
}
__device__ __forceinline__ void pair_wait(int *flag, int v) {
    while (__builtin_amdgcn_readfirstlane(__atomic_load_n(flag, __ATOMIC_RELAXED)) < v)
        __builtin_amdgcn_s_sleep(1);
}

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

// Two roles per 512-thread block, one wave of each on every SIMD (C5: 8192
// streams = 256 blocks = one per CU):
//   chain waves (threads 0..255): the per-sample loop -- NCO, mix, the newest
//     two band-edge products per lane, lane sum, powers, error, loop filter;
//   helper waves (256..511): for every chain thread, the first three products
//     of each lane accumulator, (((+0) + p0) + p1) + p2, whose inputs x[m-32],
//     x[m-24], x[m-16] are at least two blocks old: one block ahead of the
//     chain, through LDS, one s_barrier per 8-sample block.
// A lone wave issues one VALU instruction per ~5.1 cycles; two waves on a SIMD
// issue one per ~4.0 together (tools/dual_wave_probe.hip), so the helper's work
// fills issue slots the chain wave leaves empty.
__global__ __launch_bounds__(kSysThreads) void fll_sys_kernel(FllArgs a, FllParams P) {
    constexpr int N = kFllTaps;
    static_assert(N == 40, "systolic FLL assumes 5 blocks of 8 taps");
    __shared__ FllSysLds L;
    if (a.kt && threadIdx.x == 0) kt_start(a.kt);
    ClkSample clk{threadIdx.x == 0 ? a.clk : nullptr};
    if (threadIdx.x < 2 * N) L.taps[threadIdx.x] = P.lower_rev[threadIdx.x];
    if (threadIdx.x == 0) L.nmin = ~0ull;
    if (threadIdx.x < 4) L.chain_done[threadIdx.x] = L.helper_done[threadIdx.x] = 0;
    const bool helper = threadIdx.x >= kSysChain;
    const int tid = threadIdx.x & (kSysChain - 1);   // the chain thread this thread is or serves

    const int lane = tid & 63;
    const int rl = lane & 15;
    const int g = (tid >> 4) * 2 + (rl & 1);   // stream within the block
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

    __syncthreads();   // nmin initialised
    if (!helper) {
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
        if (l == 0) atomicMin(&L.nmin, static_cast<unsigned long long>(n));   // rows past S count as 0
    }
    __syncthreads();
    // blocks of the chain/helper pair loop, the same for every wave of the block:
    // samples [8, 8 + 8 NB) of every stream, with the chain's input prefetch two
    // blocks ahead still inside the shortest stream
    const int64_t nmin_blk = static_cast<int64_t>(L.nmin);
    const int64_t nb_fit = nmin_blk / 8 - 3;
    const int NB = nb_fit >= kMinPairBlocks ? static_cast<int>(nb_fit) : 0;
    typedef __attribute__((address_space(3))) f4 lds_f4;
    // 8 mixed samples x[tb .. tb+7] (tb a multiple of 8) from the ring
    auto ring_block = [&](int64_t tb, f2 *dst) __attribute__((always_inline)) {
        const lds_f4 *r = reinterpret_cast<const lds_f4 *>(ring + (tb & (kRingLen - 1)));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const f4 v = r[k];
            dst[2 * k] = f2{v.x, v.y};
            dst[2 * k + 1] = f2{v.z, v.w};
        }
    };

    if (helper) {
        if (NB > 0) {
            f2 T3[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) T3[j] = f2{L.taps[2 * (l + 8 * j)], L.taps[2 * (l + 8 * j) + 1]};
            // pair block b covers samples [8 + 8b, 16 + 8b); its step u needs
            // x[m - 32 + 8j] = sample u of blocks b-4 (j = 0), b-3, b-2 (and
            // b-1, j = 3, which the chain adds).  Block k lives in W[k mod 3].
            f2 W[3][8];
            auto emit = [&](int buf, const f2 *w0, const f2 *w1, const f2 *w2) __attribute__((always_inline)) {
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    f2 ar, ai, R, I;
                    band_prod(T3[0], w0[u], ar, ai);
                    band_prod(T3[1], w1[u], R, I);
                    ar = ar + R;
                    ai = ai + I;
                    band_prod(T3[2], w2[u], R, I);
                    ar = ar + R;
                    ai = ai + I;
                    L.part[buf][u][tid] = f4{ar.x, ar.y, ai.x, ai.y};
                }
            };
            ring_block(-24, W[2]);   // block -4
            ring_block(-16, W[0]);   // block -3
            ring_block(-8, W[1]);    // block -2
            int *cdone = &L.chain_done[tid >> 6], *hdone = &L.helper_done[tid >> 6];
            emit(0, W[2], W[0], W[1]);
            pair_publish(hdone, 1);
            if (QPSK_FLL_PROBE & 32) return;
            // iteration b: once the chain has written block b-1 (and so has read
            // P_{b-1}, whose buffer P_{b+1} takes), block b-1 -> W[(b-1) mod 3],
            // then P_{b+1} from blocks b-3, b-2, b-1
            auto it = [&](auto rc, int b) __attribute__((always_inline)) {
                constexpr int r = decltype(rc)::value;   // b mod 3
                if (b + 1 >= NB) return;
                pair_wait(cdone, b + 1);   // blocks -1 .. b-1 written
                ring_block(8 * static_cast<int64_t>(b), W[(r + 2) % 3]);
                if (!(QPSK_FLL_PROBE & 16)) emit((b + 1) & 1, W[r], W[(r + 1) % 3], W[(r + 2) % 3]);
                pair_publish(hdone, b + 2);
            };
            for (int b = 0; b < NB; b += 3) {
                it(std::integral_constant<int, 0>{}, b);
                if (b + 1 < NB) it(std::integral_constant<int, 1>{}, b + 1);
                if (b + 2 < NB) it(std::integral_constant<int, 2>{}, b + 2);
            }
        }
        return;
    }

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
#if QPSK_FLL_PROBE & 1
        } else if (true) {   // diagnostic: no sincos on the chain
            sn = phase * 0.5f;
            cs = 1.0f - phase;
#endif
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
#if QPSK_FLL_PROBE & 2
        PR = f2{0.f, 0.f}; PI = f2{0.f, 0.f};   // diagnostic: no partial-sum work
#endif
        const f2 ar = PR + R4, ai = PI + I4;
        SR = f2{shr2(SR.x) + ar.x, shr2(SR.y) + ar.y};
        SI = f2{shr2(SI.x) + ai.x, shr2(SI.y) + ai.y};
        // lane 7 holds the filter outputs of sample t: {pow upper, pow lower}
        const f2 pw = SR * SR + SI * SI;
#if QPSK_FLL_PROBE & 4
        const float err = pw.y - pw.x;   // diagnostic: no broadcast
#else
        const float err = bcast7(pw.y - pw.x, odd);
#endif
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
#if !(QPSK_FLL_PROBE & 2)
        if constexpr (decltype(reg)::value)
            partial([&](int k) -> f2 { return k == 32 ? xmv[0] : X[k]; }, u + 1);
        else
            partial(ring_at(t0), u + 1);
#endif
    };
    // 8 samples of every stream of the wave, no masks
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
        if (!(QPSK_FLL_PROBE & 8) && __builtin_expect(__ballot((amax > two_pi) | (fmx > fmax_)) != 0, 0)) {
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

    // ---- chain side of the pair loop -------------------------------------
    // Pair block b (samples t0 = 8 + 8b .. t0 + 7): the helper's 3-term partial
    // sums P_b arrive in L.part[b & 1]; the chain adds the j = 3 product with
    // x[m - 8] (block b-1, kept in registers) -- so the partial sums of every
    // step are known at the block start and kept for a redo -- then runs the 8
    // steps, writes the outputs to the ring (the helper reads them one block
    // later) and to y, and meets the helper at the barrier.
    bool need_exact = false;   // some lane's block-start phase is -0 (the shifter form excludes it)
    int *cdone = &L.chain_done[tid >> 6], *hdone = &L.helper_done[tid >> 6];
    auto cblock = [&](const f2 *in, int64_t t0, int b, const f2 *px, f2 *xo) __attribute__((always_inline)) {
        const int buf = b & 1;
        if (!(QPSK_FLL_PROBE & 32)) pair_wait(hdone, b + 1);   // P_b is in L.part[b & 1]
        f2 QR[8], QI[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const f4 v = L.part[buf][u][tid];
            f2 R3, I3;
            band_prod(TT[3], px[u], R3, I3);
            QR[u] = f2{v.x, v.y} + R3;
            QI[u] = f2{v.z, v.w} + I3;
        }
        const float ph0 = phase, fr0 = freq;
        const f2 sr0 = SR, si0 = SI;
        float amax = 0.f, fmx = 0.f;
        double umax = 0.0;
        auto core = [&](f2 inu, int u, auto exact) __attribute__((always_inline)) {
            // the chain wave is latency-bound: both polynomials side by side
            // (no lane swap), the quadrant from the shifter fma (checked by umax)
            float sn, cs;
            if constexpr (decltype(exact)::value)
                qpsk_sincosf_glibc_fast_k(phase, &sn, &cs, sign_v);
            else
                umax = fmax(umax, qpsk_sincosf_shifter_k(phase, &sn, &cs, sign_v));
            const f2 xm = add_swap_neglo(inu * f2{cs, cs}, inu * f2{sn, sn});
            xo[u] = xm;
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
        for (int u = 0; u < 8; ++u) core(in[u], u, std::false_type{});
        if (__builtin_expect(
                (__ballot((amax > two_pi) | (fmx > fmax_) | (umax > QPSK_SINCOSF_UMAX)) != 0) | need_exact, 0)) {
            // a wrap, a clamp, a quadrant near a tie or a -0 phase: redo the
            // block exactly from its start
            phase = ph0; freq = fr0; SR = sr0; SI = si0;
#pragma unroll
            for (int u = 0; u < 8; ++u) core(in[u], u, std::true_type{});
            // IEEERemainder can return -0 (an exact multiple of 2pi); a fast
            // block never creates -0 (x + y == -0 needs x == -0)
            need_exact = __ballot(__float_as_uint(phase) == 0x80000000u) != 0;
        }
        // outputs to the ring (primary slots; 64-B aligned) and to HBM
        lds_f4 *ww = reinterpret_cast<lds_f4 *>(ring + (t0 & (kRingLen - 1)));
#pragma unroll
        for (int k = 0; k < 4; ++k) ww[k] = f4{xo[2 * k].x, xo[2 * k].y, xo[2 * k + 1].x, xo[2 * k + 1].y};
#pragma unroll
        for (int u = 0; u < 8; ++u) y[t0 + u] = xo[u];
        pair_publish(cdone, b + 2);   // after the ring writes: blocks -1 .. b are in the ring
    };

    int64_t t0 = 0;
    if (NB > 0) {
        {   // the call's first block (the full sinf/cosf on its first sample), alone
            f2 cur[8];
            load8(cur, 0);
            block(cur, 0, std::true_type{});
        }
        t0 = 8;
        f2 XA[8], XB[8];   // outputs of the previous / current block, ping-pong
        ring_block(0, XB);   // block -1
        need_exact = __ballot(__float_as_uint(phase) == 0x80000000u) != 0;
        f2 A[8], B[8];
        load8(A, t0);
        load8(B, t0 + 8);
        pair_publish(cdone, 1);   // block -1 (the first block's outputs) is in the ring
        for (int b = 0; b < NB; b += 2) {
            cblock(A, t0, b, XB, XA);
            load8(A, t0 + 16);
            t0 += 8;
            if (b + 1 < NB) {
                cblock(B, t0, b + 1, XA, XB);
                load8(B, t0 + 16);
                t0 += 8;
            }
        }
        // the mirror of the last 32 samples, for the ring-window blocks that follow
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            lds_f4 *w = reinterpret_cast<lds_f4 *>(ring + ((t0 - 32 + 8 * i) & (kRingLen - 1)));
#pragma unroll
            for (int k = 0; k < 4; ++k) w[k + kRingLen / 2] = w[k];
        }
        partial(ring_at(t0), 0);
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
    hipLaunchKernelGGL(fll_sys_kernel, dim3((a.S + kSysStreams - 1) / kSysStreams), dim3(kSysThreads), 0, stream,
                       a, P);
}

}  // namespace qpsk
