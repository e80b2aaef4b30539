// qpsk_loop.hip -- symbol sync + carrier recovery + decode on gfx950.
//
// MuellerMuller.Process (MuellerMuller.cs:52-190), CostasLoopQpsk.Process
// (CostasLoopQpsk.cs:63-92), the hard decision, differential decode and
// MSB-first bit packing of QPSKDeModulator.DeModulate (QPSKDeModulator.cs:
// 364-408).  Both loops are serial recurrences per stream, so a stream's work
// cannot be spread over lanes; measured on MI355X (tools/dep_probe.hip) one
// wave issues one instruction per ~4 cycles, dependent or not, so a chain's
// time per symbol is its instruction count x 4 plus its LDS round trips, and
// the lever is to give each stage of a stream its OWN wave (its own SIMD issue
// port) and keep memory off the chains:
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
#include <type_traits>

#include "qpsk_glibc_trig.h"
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

// KB = samples per round per stream (template: 64 or 128).  The per-stream
// sample ring holds 4 rounds (index = p & (4*KB - 1)), preceded by a mirror of
// its last 4 samples so the 4 interpolation taps are always contiguous in LDS.
constexpr int kMir = 4;
template <int KB> struct Ring {
    static constexpr int len = 4 * KB;
    static constexpr int row = kMir + len;   // per-stream LDS row: [mirror 4][ring]
};
// symbols per round per stream (template CAP): at most floor((KB + 3) / (sps - 0.1)) + 1
// start in one round: 75 (KB 64, sps >= 1), 36 (KB 64, sps >= 2), 69 (KB 128, sps >= 2)
constexpr int kCapAny = 80;
constexpr int kCapSps2 = 40;
constexpr int kCap128Sps2 = 72;
// sps >= 4 / >= 8: the same backlog limit (lag_max = KB/2) with fewer symbol
// slots, so the workgroup's LDS drops from 143.5 KB to 125 KB / 104 KB and a
// matched-filter workgroup of the next pipelined call fits beside it
constexpr int kCapSps4 = 28;
constexpr int kCapSps8 = 14;
// 128-sample rounds at sps >= 8 (variant 4): lag_max = 64 needs
// (CAP - 1)(sps - 0.1) >= KB + 4 + 64 -> CAP = 26
constexpr int kCap128Sps8 = 26;
// 256-sample rounds at sps >= 8 (variant 6): lag_max = 128 needs
// (CAP - 1)(sps - 0.1) >= KB + 4 + 128 -> CAP = 51
constexpr int kCap256Sps8 = 51;
// 512-sample rounds at sps >= 8 (variant 7): lag_max = 256 needs CAP >= 99;
// 100 makes the row stride (CAP + 1) odd
constexpr int kCap512Sps8 = 100;
typedef double d2 __attribute__((ext_vector_type(2)));

// M&M -> Costas symbol slots.  64-sample rounds (the 32 x 64 shapes of C3, C4
// and C5): the M&M's float symbols, which the Costas wave widens (exactly);
// the M&M's store halves (ds_write_b64), and with the M&M pacing these shapes
// the loop runs faster: C3 331.7 -> 318.0 and C4 396.9 -> 377.5 cycles per
// symbol, A/B x2 on one MI355X (profiles/r06_float_slots_ab.txt).  Longer
// rounds (C2's 6 x 512, 12 x 256, 24 x 128), where the Costas wave paces and
// the two widenings land on it: the doubles the M&M already has (C2 274 ->
// 291 with float slots).  Round 2 measured float slots slower at C3 when the
// Costas wave still paced there.
typedef d2 sym_t;
__device__ __forceinline__ d2 from_sym(d2 v) { return v; }
__device__ __forceinline__ d2 from_sym(f2 v) { return d2{static_cast<double>(v.x), static_cast<double>(v.y)}; }
template <typename S> struct SymPut;
template <> struct SymPut<d2> {
    __device__ static d2 put(float, float, double cid, double cqd) { return d2{cid, cqd}; }
};
template <> struct SymPut<f2> {
    __device__ static f2 put(float ci, float cq, double, double) { return f2{ci, cq}; }
};
// (the glibc-trig Costas step paces its loop at every shape: doubles there)
template <int KB, int TRIG>
using SymSlot = typename std::conditional<KB == 64 && TRIG == 0, f2, d2>::type;

__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int w = __shfl_xor(v, o, 64);
        v = w > v ? w : v;
    }
    // every lane holds the maximum now; readfirstlane tells the compiler so,
    // which keeps loops bounded by it scalar (no exec-mask loop control)
    return __builtin_amdgcn_readfirstlane(v);
}

// r of the lower half (lanes 0-31) and of the upper half (lanes 32-63) of the
// wave, each into every lane: v_permlane32_swap exchanges the upper half of
// its first operand with the lower half of its second (lo and hi dwords)
__device__ __forceinline__ void swap_halves(double r, double *lower, double *upper) {
    const uint64_t b = __builtin_bit_cast(uint64_t, r);
    const uint32_t lo = static_cast<uint32_t>(b), hi = static_cast<uint32_t>(b >> 32);
    const auto pl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto ph = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    *lower = __builtin_bit_cast(double, (static_cast<uint64_t>(ph[0]) << 32) | pl[0]);
    *upper = __builtin_bit_cast(double, (static_cast<uint64_t>(ph[1]) << 32) | pl[1]);
}

// x or -x, i.e. x times +1.0 or -1.0 exactly: one v_cndmask_b32 with a
// negated source on the high word.  The high word is made opaque as a float,
// so the select keeps its fneg as a source modifier instead of becoming an
// xor; in place when x dies at the select
__device__ __forceinline__ double signsel(double x, bool pos) {
    const uint64_t b = __builtin_bit_cast(uint64_t, x);
    float h = __builtin_bit_cast(float, static_cast<uint32_t>(b >> 32));
    asm("" : "+v"(h));
    const float r = pos ? h : -h;
    return __builtin_bit_cast(double, (static_cast<uint64_t>(__builtin_bit_cast(uint32_t, r)) << 32) |
                                          static_cast<uint32_t>(b));
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

// Symbol rows are CAP + 1 entries long: an odd stride puts the 32 streams'
// entry k (read by all lanes at once in the Costas loop) on distinct banks;
// a stride of 40 made them 16- to 32-way bank conflicts.
template <int CAP>
struct RowStride { static constexpr int value = CAP + 1; };

// TRIG 0: the portable sincos table (qpsk_sincos.h), heads and tails; TRIG 1:
// glibc's __sincostab in the split form's two layouts (qpsk_glibc_trig.h:
// do_sin rows at 0, do_cos rows at 440), no tails
// ROTB: the Costas wave hands the decode wave only the two decisions (the
// sign bytes of +-1.0, 2 B per symbol) instead of the rotated symbol (8 B)
// when no symbols are written out: at C3 the workgroup drops from 125 KB to
// 114 KB of LDS, and two matched-filter workgroups of the next pipelined
// call fit beside it instead of one
template <int SPW, int CAP, int KB, int TRIG, bool ROTB>
struct LoopLds {
    static constexpr int RS = RowStride<CAP>::value;
    double tab[TRIG ? 880 : 1024];  // sincos table head, at LDS offset 0 so
    double tab_lo[TRIG ? 2 : 1024]; // the table index is the whole address; tail (floats, widened)
    // the symbol slots sit below 64 KB, ahead of the ring: a ds instruction's
    // immediate offset is 16 bits, so the Costas wave's per-step slot reads and
    // writes then fold their constant part into the instruction instead of one
    // v_add_u32 each (behind the 66 KB ring they did)
    SymSlot<KB, TRIG> sym[2 * SPW * RS];   // M&M -> Costas [slot][stream][RS] (see SymSlot)
    typename std::conditional<ROTB, uint16_t, f2>::type rot[2 * SPW * RS];   // Costas -> decode
    int cnt[4 * SPW + 4];          // symbols produced by the M&M in round r: cnt[r & 3];
                                   // cnt[4*SPW + (r & 3)] = their minimum over the batch
    alignas(16) f2 mf[SPW * Ring<KB>::row];   // sample ring [stream][mirror | 4 rounds x KB]
};

// SPW = streams (LDS rows) per workgroup; ACT >= SPW = lanes of the stage
// waves that run the chains: lanes SPW <= l < ACT shadow the workgroup's first
// stream on its own LDS rows (same addresses as lane 0, same values written),
// so a shape with few rows (long rounds) still keeps its waves' lanes busy
template <int MODE, bool DIFF, bool SYMS, int SPW, int CAP, int KB, int TRIG, int ACT>
__global__ __launch_bounds__(256) void loop_kernel(LoopArgs a, LoopParams P) {
    static_assert(ACT >= SPW && ACT <= (TRIG ? 32 : 64), "active lanes");
    constexpr int kRing = Ring<KB>::len, kRowS = Ring<KB>::row;
    // one LDS object only: a second __shared__ object would make hipcc drain the
    // loader's LDS-DMA before touching it (cdna_hip_programming.md §5)
    constexpr bool ROTB = !SYMS;
    __shared__ LoopLds<SPW, CAP, KB, TRIG, ROTB> L;

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    if (wave == 1 && lane == 0) {
        if (a.kt) kt_start(a.kt);
        // this workgroup holds its CU now: the next pipelined call's FIR waits
        // for min(grid, CUs) of these (qpsk_runtime.hip, process_async_one)
        if (a.resident) __hip_atomic_fetch_add(a.resident, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // the stage waves record the launch end as they leave (not the loader, whose
    // vmcnt waits count its own outstanding memory operations)
    KtEnd kte{wave != 0 ? a.kt : nullptr};
    ClkSample clk{wave == 1 && lane == 0 ? a.clk : nullptr};
    // FIR phase sample: this workgroup's CU is counted while its M&M wave runs
    // (a count, not a flag: two loop workgroups may share a CU, and the first
    // to leave must not clear the other's mark)
    struct CuMark {
        unsigned *p;
        __device__ explicit CuMark(unsigned *map) : p(map ? map + cu_key() : nullptr) {
            if (p) __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __device__ ~CuMark() {
            if (p) __hip_atomic_fetch_sub(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    } cu_mark{wave == 1 && lane == 0 ? a.cu_map : nullptr};
    // the batch spread evenly over the grid: workgroup b owns streams
    // [b S / G, (b + 1) S / G), at most SPW.  A workgroup left with few
    // streams (e.g. 16 of 24 at S = 256) runs its uniform loops ~10-25 %
    // slower per symbol than a full one, and the kernel waits for it
    const int blk_s0 = static_cast<int>(static_cast<int64_t>(blockIdx.x) * a.S / gridDim.x);
    const int nvalid = static_cast<int>(static_cast<int64_t>(blockIdx.x + 1) * a.S / gridDim.x) - blk_s0;
    const int s = blk_s0 + lane;
    // lanes SPW > l >= nvalid shadow the workgroup's first stream: they run its
    // M&M and Costas chains too (on the copy of its samples the loader puts in
    // their ring rows) and write nothing.  A wave with 16 or fewer active lanes
    // runs these loops 10-50 % slower per symbol than one with 20 or more
    // (profiles/archive/r02_loop_probe_lanes.txt), so small batches keep SPW lanes busy
    const bool real = lane < nvalid;            // owns stream s: writes its results
    const bool valid = lane < ACT;              // computes stream sc
    const int sc = real ? s : blk_s0;
    const int rowl = lane < SPW ? lane : 0;     // LDS row of stream sc

    // ---- per-stream queue geometry (every wave: lane l <-> stream sc)
    int n = 0, cnt = 0, R = 0, d = 0;
    if (valid) {
        n = static_cast<int>(a.lengths ? a.lengths[sc] : a.n);
        R = a.state[sc].carry_n;
        d = R & 1;
        cnt = R + d + n;
        // DeModulate with an empty span returns before touching any state (:350-351)
        if (MODE == kModeDemodulate && n == 0) cnt = 0;
    }
    const int NR = (wave_max_i32(cnt) + KB - 1) / KB;
    const bool mine = valid && cnt > 0;

    if constexpr (TRIG) {
        for (int i = threadIdx.x; i < 110; i += 256)
            qpsk_gl_half_tables(qpsk_gl_sincostab_dev, i, L.tab + 4 * i, L.tab + 440 + 4 * i);
    } else {
        for (int i = threadIdx.x; i < 1024; i += 256) {
            L.tab[i] = qpsk_sincos_table_dev[i];
            L.tab_lo[i] = qpsk_sincos_table_dev_lo[i];
        }
    }
    __syncthreads();

#ifdef QPSK_LOOP_STAMPS
    if (a.probe && lane == 0) {   // where each wave runs: HW_ID (SIMD, CU, SE) and XCC
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
        a.probe[blockIdx.x * 16 + 12 + wave] = hw | (static_cast<unsigned long long>(xcc) << 32);
    }
#endif
    if (wave == 0) {
        // ============================================================ loader
        // one glds instruction = KB/2 lanes x 16 B = one stream's round (8*KB
        // bytes); KB = 256: NI = 2 instructions of 64 lanes (128 samples each)
        constexpr int NI = KB > 128 ? KB / 128 : 1;
        const int64_t org = valid ? sc * a.mf_stride + kMfPrefix - R - d : 0;
        const int c2 = 2 * (lane % (KB / 2 < 64 ? KB / 2 : 64));
        const f2 *mf = reinterpret_cast<const f2 *>(a.mf);
        const bool lo_half = lane < KB / 2;
        // Fast path (every round but a stream's last): byte offsets of each
        // stream's queue relative to the workgroup's first MF row, computed once
        // and kept in VGPRs, so a round costs one SGPR base update plus, per
        // stream, M0 + one global_load_lds (no per-stream readlanes or bounds
        // tests).  Rows past the batch reuse stream 0's offsets (in bounds).
        const f2 *wg_mf = mf + static_cast<int64_t>(blk_s0) * a.mf_stride;
        uint32_t voff[SPW];
#pragma unroll
        for (int j = 0; j < SPW; ++j) {
            const int jj = j < nvalid ? j : 0;
            const int64_t oj = readlane64(org, jj) - static_cast<int64_t>(blk_s0) * a.mf_stride;
            voff[j] = static_cast<uint32_t>((oj + c2) * 8);
        }
        // the fast path needs every stream of the workgroup to hold the whole round
        int cmin = valid ? cnt : 0x7fffffff;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const int w = __shfl_xor(cmin, o, 64);
            cmin = w < cmin ? w : cmin;
        }
        cmin = __builtin_amdgcn_readfirstlane(cmin);
        auto issue = [&](int r) {
            const int roff = (r & 3) * KB;
            if ((r + 1) * KB <= cmin) {
                const char *rb = reinterpret_cast<const char *>(wg_mf + static_cast<int64_t>(r) * KB);
#pragma unroll
                for (int j = 0; j < SPW; ++j)
#pragma unroll
                    for (int h = 0; h < NI; ++h)
                        if (lo_half)
                            __builtin_amdgcn_global_load_lds((glb_void_t *)(rb + voff[j] + 1024 * h),
                                                             (lds_void_t *)(L.mf + j * kRowS + kMir + roff + 128 * h),
                                                             16, 0, 0);
                return;
            }
#pragma unroll 4
            for (int j = 0; j < SPW; ++j) {
                const int c = __builtin_amdgcn_readlane(cnt, j);
                const int64_t o = readlane64(org, j);
#pragma unroll
                for (int h = 0; h < NI; ++h) {
                    int p = r * KB + c2 + 128 * h;
                    // past the stream's end: read a harmless in-row pair (never used);
                    // a pair straddling the end reads one sample of row slack
                    if (p >= c) p = 0;
                    if (lo_half)
                        __builtin_amdgcn_global_load_lds((glb_void_t *)(mf + o + p),
                                                         (lds_void_t *)(L.mf + j * kRowS + kMir + roff + 128 * h),
                                                         16, 0, 0);
                }
            }
        };
#ifdef QPSK_LOOP_STAMPS
        unsigned long long t_wait = 0, t_bar = 0, t_issue = 0;
#endif
        if (NR > 0) issue(0);
        if (NR > 1) issue(1);
        for (int r = 0; r <= NR + 1; ++r) {
            STAMP(ta);
            // round r's loads done, round r + 1's (SPW * NI, the counter holds 63) in flight
            if (r + 1 < NR) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(SPW * NI < 63 ? SPW * NI : 63) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            ACC(t_wait, ta);
            STAMP(tb);
            __builtin_amdgcn_s_barrier();
            ACC(t_bar, tb);
            STAMP(ti);
            if (r + 2 < NR) issue(r + 2);
            ACC(t_issue, ti);
        }
#ifdef QPSK_LOOP_STAMPS
        if (a.probe && lane == 0) {
            a.probe[blockIdx.x * 16 + 0] = t_wait;
            a.probe[blockIdx.x * 16 + 1] = t_bar + (t_issue << 32);
        }
#endif
        return;
    }

    if (wave == 1) {
        // ============================================================ M&M
        StreamState st;
        if (mine) st = a.state[sc];
        int base = mine ? st.base + d : 0;          // physical baseIndex
        double mu = st.mu, integ = st.integ;
        float psi = st.psi, psq = st.psq, pdi = st.pdi, pdq = st.pdq;
        int has_prev = mine ? st.has_prev : 1;
        const double sps = P.sps, kp = P.kp, ki = P.ki;
        // the clamp bounds pinned in VGPRs: as SGPR pairs the compiler rebuilt
        // -0.1 from 0.1's low word with an s_mov every symbol
        double clamp_hi = 0.1, clamp_lo = -0.1;
        asm volatile("" : "+v"(clamp_hi), "+v"(clamp_lo));
        const int cap = n;                          // output span = 2n floats (QPSKDeModulator.cs:366)
        int nsym = 0;
        bool stop = !mine;                          // capacity reached (MuellerMuller.cs:101-102)
        f2 *row = L.mf + rowl * kRowS;
        // taps x[b-1..b+2] of physical index b: contiguous thanks to the mirror
        auto taps = [&](int b) -> const f2 * { return row + kMir - 3 + ((b + 2) & (kRing - 1)); };
        // Timing runs in the reference's coordinates: t = baseIndex + mu with
        // baseIndex counted from the start of the whole DeModulate call's queue
        // (MuellerMuller.cs:113-115 rounds newTime at that magnitude).  P = the
        // queue index of this chunk's first sample (0 unless the call was split
        // into internal chunks); physical index b = floor(t) - P + d.
        const int P = mine ? static_cast<int>(st.tofs) : 0;
        const int dP = d - P;
        // the same address straight from floor(t): fl + (1.5*2^52 + dP + 2) holds
        // b + 2 in its low mantissa bits (no float->int conversion on the chain)
        const double tap_shift = 6755399441055744.0 + static_cast<double>(dP + 2);
        // loop-invariant LDS address of x[-3] relative to the ring, kept opaque so
        // the whole base lives in one VGPR and the tap reads use immediate offsets
        typedef __attribute__((address_space(3))) const f2 lds_f2;
        uint32_t tap0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_f2 *)(row + kMir - 3)));
        asm volatile("" : "+v"(tap0));
        auto taps_fl = [&](double fl) -> lds_f2 * {
            union { double v; unsigned long long u; } kb;
            kb.v = fl + tap_shift;
            // and + lshl_add: one op shorter than the shift, and, add the
            // compiler canonicalises 8 * (i & m) + base into
            const uint32_t idx = static_cast<uint32_t>(kb.u) & (kRing - 1);
            uint32_t addr;
            asm("v_lshl_add_u32 %0, %1, 3, %2" : "=v"(addr) : "v"(idx), "v"(tap0));
            return reinterpret_cast<lds_f2 *>(static_cast<uintptr_t>(addr));
        };
        // symbols that start in every 64-sample round once a stream is inside its
        // samples: the timing advance is at most sps + 0.1 per symbol
        const int kguar = __builtin_amdgcn_readfirstlane(static_cast<int>(floor((KB - sps - 4.0) / (sps + 0.1))));
        // the per-round votes' thresholds (G - 1) * step_max, G = kguar .. kguar + 3
        const double step_max = sps + 0.1;
        const double thr0 = (kguar - 1) * step_max, thr1 = kguar * step_max;
        const double thr2 = (kguar + 1) * step_max, thr3 = (kguar + 2) * step_max;
        // largest backlog (samples behind rend) a stream may carry into the next
        // round: half a round keeps its taps inside the ring slots not being
        // refilled, and a round then holds at most (KB + lag_max + 4)/(sps - 0.1) + 1
        // <= CAP symbols; <= 0 (small sps) means every round is finished
        const double lag_max = fmin(0.5 * KB, (CAP - 1) * (sps - 0.1) - KB - 4.0);
        // logical time baseIndex + mu.  After baseIndex = floor(t), mu = t - baseIndex
        // (exact, Sterbenz), (double)baseIndex + mu == t exactly, so the reference's
        // next time baseIndex + mu + advance (MuellerMuller.cs:113) is simply t + advance
        double nt = static_cast<double>(base - dP) + mu;
        // the TED reuses the previous symbol widened to double and the decisions
        // as doubles +-1.0: d*x is exact, so fma(d1, x1, d2*x2) rounds the same
        // exact sum as the reference's (double)d1*x1 + (double)d2*x2
        double psid = psi, psqd = psq;
        double pdid = pdi >= 0.0f ? 1.0 : -1.0, pdqd = pdq >= 0.0f ? 1.0 : -1.0;
#ifdef QPSK_LOOP_STAMPS
        unsigned long long c_bar = 0, c_loop = 0, c_iters = 0, c_uni = 0, c_uit = 0, c_pre = 0, c_post = 0;
#endif
        for (int r = 0; r <= NR + 1; ++r) {
            STAMP(tb);
            __builtin_amdgcn_s_barrier();
            ACC(c_bar, tb);
            if (r >= NR) continue;
            STAMP(tl);
            if ((r & 3) == 0 && r > 0 && mine && lane < SPW) {
                // mirror = last 4 samples of the ring (round r-1, already consumed)
                row[0] = row[kMir + kRing - 4]; row[1] = row[kMir + kRing - 3];
                row[2] = row[kMir + kRing - 2]; row[3] = row[kMir + kRing - 1];
            }
            const int rend = (r + 1) * KB < cnt ? (r + 1) * KB : cnt;
            auto *out = L.sym + ((r & 1) * SPW + rowl) * L.RS;
            int kmax = stop ? 0 : (cap - nsym < CAP ? cap - nsym : CAP);
            int k = 0, kuni = 0;
            lds_f2 *tp = (lds_f2 *)taps(base);
            f2 xm1 = tp[0], x0 = tp[1], x1 = tp[2], x2 = tp[3];
            // CubicLagrange4 (MuellerMuller.cs:160-190), float
            auto interp = [&](float &ci, float &cq) {
                const float t = static_cast<float>(mu);
                // the reference's products, two per packed op:
                //   cm1 = -((t*tm1)*tm2)/6  c0 = ((tp1*tm1)*tm2)/2
                //   c1 = -((tp1*t)*tm2)/2   c2 = ((tp1*t)*tm1)/6
                // (-x)*c == x*(-c) bit for bit, so the negations ride on the
                // constants; t + 0 == t (t = (float)mu is +0 or positive or NaN)
                const f2 p1 = f2{t, t} + f2{0.0f, 1.0f};       // {t, tp1}
                const f2 p2 = f2{t, t} + f2{-2.0f, -1.0f};     // {tm2, tm1}
                const f2 bd = (p1 * p2.y) * p2.x;
                const f2 fg = p2 * (p1.y * p1.x);
                const f2 c01 = bd * f2{-(1.0f / 6.0f), 1.0f / 2.0f};
                const f2 c23 = fg * f2{-(1.0f / 2.0f), 1.0f / 6.0f};
                // ((cm1*xm1 + c0*x0) + c1*x1) + c2*x2 for I and Q in one packed op each
                const f2 acc = ((c01.x * xm1 + c01.y * x0) + c23.x * x1) + c23.y * x2;
                ci = acc.x;
                cq = acc.y;
            };
            // advance timing by adv (MuellerMuller.cs:113-115) and fetch the next taps
            // LOAD = false: a round's last uniform step fetches no taps; they
            // would be stale (samples of the next round) and the round-start
            // reload would first have to wait for them
            auto advance = [&](double adv, auto load) {
                nt = nt + adv;
                const double fl = floor(nt);
                mu = nt - fl;
                base = static_cast<int>(fl) + dP;
                if constexpr (decltype(load)::value) {
                    tp = taps_fl(fl);
                    xm1 = tp[0]; x0 = tp[1]; x1 = tp[2]; x2 = tp[3];
                    // the tap loads go out before anything after them in the
                    // source (the step's symbol store, the next interpolation's
                    // coefficients), which then runs under their LDS round trip
                    __builtin_amdgcn_sched_barrier(0);
                }
            };
            auto reload = [&]() {
                tp = (lds_f2 *)taps(base);
                xm1 = tp[0]; x0 = tp[1]; x1 = tp[2]; x2 = tp[3];
            };
            if (!has_prev && base + 2 < rend && kmax > 0) {
                // very first symbol of the stream: no TED, advance = sps (MuellerMuller.cs:93-97)
                float ci, cq;
                interp(ci, cq);
                has_prev = 1;
                psid = ci; psqd = cq;
                out[k++] = SymPut<SymSlot<KB, TRIG>>::put(ci, cq, psid, psqd);
                psi = ci; psq = cq;
                pdid = ci >= 0.0f ? 1.0 : -1.0;
                pdqd = cq >= 0.0f ? 1.0 : -1.0;
                advance(sps, std::true_type{});
            }
            auto step = [&](auto load) {
                float ci, cq;
                interp(ci, cq);
                // M&M TED (MuellerMuller.cs:78-80)
                const double did = ci >= 0.0f ? 1.0 : -1.0;
                const double dqd = cq >= 0.0f ? 1.0 : -1.0;
                const double cid = ci, cqd = cq;
                // (dq * x as a sign select, signsel, measured one instruction
                // longer here: the copy it needs of cqd's low word, twice)
                const double t1 = fma(pdid, cid, pdqd * cqd);
                const double t2 = fma(did, psid, dqd * psqd);
                const double e = t1 - t2;
                // PI filter, clamp, advance (MuellerMuller.cs:83-91)
                integ = integ + ki * e;
                const double c = kp * e + integ;
                // the clamp as min/max: c > 0.1 -> 0.1, c < -0.1 -> -0.1 (a NaN c,
                // which the reference cannot survive either, clamps instead of
                // propagating)
                const double corr = __builtin_fmax(__builtin_fmin(c, clamp_hi), clamp_lo);
                psid = cid; psqd = cqd;
                pdid = did; pdqd = dqd;
                advance(sps + corr, load);
                // stored after the next taps' loads (LDS serves in issue order)
                out[k++] = SymPut<SymSlot<KB, TRIG>>::put(ci, cq, cid, cqd);
#ifdef QPSK_LOOP_STAMPS
                ++c_iters;
#endif
            };
            // Symbols K = 0..G-1 of this round are certain to start while
            // t + K (sps + 0.1) + d + 3 <= rend (the advance is at most sps + 0.1;
            // one sample of margin absorbs rounding) and capacity allows.  Votes
            // on the likely counts let the wave run the largest count every live
            // stream reaches as a uniform loop (no per-lane exit masks).  A stream
            // need not finish its round: what it leaves (its backlog) stays in the
            // ring and opens the next round, so the wave-wide count settles at
            // the symbol rate and no per-lane remainder runs in steady state.
            {
                const double room = static_cast<double>(rend - dP - 3) - nt;
                const int cap_l = kmax - k;
                // streams whose samples end in this round vote too; streams that
                // ended earlier, stopped ones and rows past the batch do not
                const bool live = mine & !stop & (cnt > r * KB);
                // reaches(G) = room >= (G - 1) step_max and cap_l >= G, i.e.
                // (G - 1) step_max <= eff = min(room, (cap_l - 1) step_max): the
                // rounded products of distinct small integers with step_max keep
                // their order.  Non-voters hold +inf.  Each vote is then one
                // v_cmp straight into an SGPR mask, and the count is picked with
                // scalar selects (no VALU <-> SALU round trip per vote)
                const double eff = live ? __builtin_fmin(room, (cap_l - 1) * step_max) : __builtin_inf();
                int kg = 0;
                const uint64_t m0 = __builtin_amdgcn_ballot_w64(!(eff >= thr0));
                const uint64_t m1 = __builtin_amdgcn_ballot_w64(!(eff >= thr1));
                const uint64_t m2 = __builtin_amdgcn_ballot_w64(!(eff >= thr2));
                const uint64_t m3 = __builtin_amdgcn_ballot_w64(!(eff >= thr3));
                kg = m2 == 0 ? (m3 == 0 ? kguar + 3 : kguar + 2)
                             : (m1 == 0 ? kguar + 1 : (m0 == 0 ? kguar : 0));
                kg = __builtin_amdgcn_readfirstlane(kg);
                kuni = kg > 0 ? kg : 0;
                ACC(c_pre, tl);
                STAMP(tu);
                if (live) {
                    // an even unroll: the loop-carried symbol/decision registers
                    // alternate instead of being copied back every symbol
                    int u = 0;
                    // by four: a lone wave pays ~28 cycles per taken loop branch
                    // (tools/dep_probe.hip), 7 per symbol instead of 14.  C2 loop
                    // 18.4 -> 17.3 ms (326 -> 306 cycles per symbol, A/B x2 on one
                    // MI355X, profiles/r05_loop_unroll4_ab.txt); C3 / C4 unchanged
                    for (; u + 4 < kg; u += 4) {
                        step(std::true_type{});
                        step(std::true_type{});
                        step(std::true_type{});
                        step(std::true_type{});
                    }
                    if (kg - u >= 4) step(std::true_type{});
                    if (kg - u >= 3) step(std::true_type{});
                    if (kg - u >= 2) step(std::true_type{});
                    if (kg - u >= 1) step(std::false_type{});
                }
                ACC(c_uni, tu);
#ifdef QPSK_LOOP_STAMPS
                c_uit += kuni;
#endif
            }
            STAMP(tpost);
            // per-lane catch-up: a stream's last round finishes it; before that
            // it steps on only while it lags rend by lag_max samples or more,
            // which bounds the backlog (ring and round capacity stay safe).
            // k < kmax also bounds a stream whose timing went NaN (base stuck)
            {
                const bool last = cnt <= (r + 1) * KB;
                auto more = [&]() {
                    return (base + 2 < rend) & (k < kmax) &
                           (last | (static_cast<double>(rend - dP - 3) - nt >= lag_max));
                };
                if (__builtin_amdgcn_ballot_w64(more()) != 0) {   // one vote skips the loop in steady state
                    reload();                   // the uniform loop ended on a tap-less step
                    while (more()) step(std::true_type{});
                }
            }
            nsym += k;
            if (!stop && nsym >= cap && base + 2 < rend) {
                // MuellerMuller.cs:73-102: the symbol after the last one that fits
                // still runs the TED/PI update, then the call stops
                reload();
                float ci, cq;
                interp(ci, cq);
                const float di = ci >= 0.0f ? 1.0f : -1.0f;
                const float dq = cq >= 0.0f ? 1.0f : -1.0f;
                if (has_prev) {   // psid/psqd/pdid/pdqd hold the floats exactly
                    const double t1 = pdid * ci + pdqd * cq;
                    const double t2 = static_cast<double>(di) * psid + static_cast<double>(dq) * psqd;
                    integ += ki * (t1 - t2);
                }
                has_prev = 1;
                stop = true;
            }
            // the Costas wave runs the uniform count as its own uniform loop on
            // every stream that produced at least that many symbols
            if (lane < SPW) L.cnt[(r & 3) * SPW + lane] = k;
            if (lane == 0) L.cnt[4 * SPW + (r & 3)] = kuni;
            ACC(c_post, tpost);
            ACC(c_loop, tl);
        }
#ifdef QPSK_LOOP_STAMPS
        if (a.probe && lane == 0) {
            a.probe[blockIdx.x * 16 + 2] = c_bar;
            a.probe[blockIdx.x * 16 + 3] = c_loop;
            a.probe[blockIdx.x * 16 + 4] = c_iters | (c_uni << 20);
            a.probe[blockIdx.x * 16 + 7] = NR;
            a.probe[blockIdx.x * 16 + 10] = c_uit;
            a.probe[blockIdx.x * 16 + 11] = c_pre + (c_post << 32);
        }
#endif
        if (!real) return;
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
            if (a.flags) atomicOr(a.flags, 1u);
            consumed = count - kCarryMax;
            keep = kCarryMax;
        }
        // a non-finite sample that reached the timing loop leaves the PI
        // integrator NaN: the reference's correction, and with it newTime, go
        // NaN, and (int)Math.Floor(NaN) = 0 (.NET 9 saturating conversion) pins
        // baseIndex at 0 from then on (MuellerMuller.cs:83-115).  This kernel
        // clamps the NaN correction instead; the call is flagged either way.
        if (!(integ == integ) && a.flags) atomicOr(a.flags, 4u);
        const f2 *q = reinterpret_cast<const f2 *>(a.mf) + s * a.mf_stride + kMfPrefix - R;  // logical 0
        f2 *cw = reinterpret_cast<f2 *>(a.carry) + static_cast<int64_t>(s) * kCarryMax;
        for (int i = 0; i < keep; ++i) cw[i] = q[consumed + i];
        StreamState *g = a.state + s;
        g->base = lbase - consumed;
        g->carry_n = keep;
        g->tofs = a.chunked ? static_cast<int64_t>(P) + consumed : 0;
        g->mu = mu;
        g->integ = integ;
        // the widened registers hold the reference's floats exactly
        psi = static_cast<float>(psid);
        psq = static_cast<float>(psqd);
        pdi = static_cast<float>(pdid);
        pdq = static_cast<float>(pdqd);
        g->psi = psi; g->psq = psq; g->pdi = pdi; g->pdq = pdq;
        g->has_prev = has_prev;
        return;
    }

    if (wave == 2) {
        // ============================================================ Costas
        // TRIG 1: lanes l and l + 32 both run stream l (SPW <= 32), for the split
        // glibc sincos: the lower lane evaluates the do_sin, the upper the do_cos
        // (qpsk_glibc_trig.h), and v_permlane32_swap hands each its partner's
        // result; both halves then run the same Costas update
        const int cl = TRIG ? (lane & 31) : lane;
        const bool cmine = TRIG ? (__shfl(mine ? 1 : 0, cl, 64) != 0) : mine;
        const int csc = TRIG ? __shfl(sc, cl, 64) : sc;
        const int half = TRIG ? (lane >> 5) : 0;
        const double *tabh = L.tab + (half ? 440 : 0);
        // fast-split lane constants: the lower half runs do_sin, the upper do_cos
        qpsk_gl_fs_lane KF = qpsk_gl_fs_lane_init(half == 0);
        asm volatile("" : "+v"(KF.L0), "+v"(KF.L1), "+v"(KF.hp1L), "+v"(KF.sgnm), "+v"(KF.tsh), "+v"(KF.sign));
        asm volatile("" : "+v"(KF.toint), "+v"(KF.s4), "+v"(KF.sn3), "+v"(KF.cs4));
        double theta = 0.0, freq = 0.0;
        if (cmine) {
            theta = a.state[csc].theta;
            freq = a.state[csc].freq;
        }
        double ca = P.c_alpha, cb = P.c_beta;
        double kTwoPi = 2.0 * 3.14159265358979311600;
        double kPi = 3.14159265358979311600;
        qpsk_sincos_consts K = QPSK_SINCOS_CONSTS_INIT;
        // every 64-bit constant of the step lives in VGPRs for the whole wave:
        // otherwise each iteration rebuilds some from SGPR halves (VOP3 reads
        // one scalar operand), which costs issue slots on an issue-bound chain
        asm volatile("" : "+v"(ca), "+v"(cb), "+v"(kTwoPi), "+v"(kPi));
        asm volatile("" : "+v"(K.INV), "+v"(K.SH), "+v"(K.P1), "+v"(K.P2));
        asm volatile("" : "+v"(K.S3), "+v"(K.S5), "+v"(K.C4), "+v"(K.C6));
#ifdef QPSK_LOOP_STAMPS
        unsigned long long k_bar = 0, k_loop = 0, k_uni = 0, k_uit = 0;
#endif
        for (int r = 0; r <= NR + 1; ++r) {
            STAMP(tb);
            __builtin_amdgcn_s_barrier();
            ACC(k_bar, tb);
            if (r == 0 || r > NR) continue;
            STAMP(tl);
            const int slot = (r - 1) & 1;
            const int mlo = __builtin_amdgcn_readfirstlane(L.cnt[4 * SPW + ((r - 1) & 3)]);
            if (cl >= ACT) continue;   // exec = the batch's lanes for the whole round
            const int crow = cl < SPW ? cl : 0;
            const int m = cmine ? L.cnt[((r - 1) & 3) * SPW + crow] : 0;
            const auto *in = L.sym + (slot * SPW + crow) * L.RS;
            // (TRIG 1: both lanes of a stream store the same value to the same slot)
            auto *out = L.rot + (slot * SPW + crow) * L.RS;
            d2 y;
            // CostasLoopQpsk.cs:63-92: double NCO, float I/O (y widened to double).
            // HUGE: theta may exceed the table reduction's range (|theta| <= 2^40,
            // qpsk_sincos_arg); the fast pass assumes it does not and the round is
            // redone if it did.  Below 2^40 the fast pass is exact: a stream in a
            // QPSK false lock (|freq| > pi, theta growing every symbol) keeps the
            // fast path for ~10^5 calls (profiles/archive/r02_state_c3.log: a 4096-stream
            // C3 batch has 27 such streams after 6 calls; with the old 1e6 range
            // their 26 workgroups redid every round and the kernel took 2.7x)
            auto widen = [](SymSlot<KB, TRIG> v) { return from_sym(v); };
            // the previous step's decisions, stored under this step's table loads
            // (row entry CAP, past the round's symbols, takes the first store)
            typename std::remove_reference<decltype(out[0])>::type pend{};
            int pend_k = CAP;
            double amax = fabs(theta);   // largest sincos argument of the round
            auto track = [&]() { asm volatile("v_max_f64 %0, %0, |%1|" : "+v"(amax) : "v"(theta)); };
            auto step = [&](int k, auto huge) {
                double sn, cs;
                // Math.Sin/Cos = glibc; the fast pass leaves its Payne-Hanek reduction out
                if constexpr (TRIG && !decltype(huge)::value) {
                    // the fast pass: the pair of |theta| (qpsk_glibc_trig.h, fast split form)
                    int sw;
                    const double rh = qpsk_gl_fs_pair(theta, &KF, tabh, &sw);
                    double VS, VC;
                    swap_halves(rh, &VS, &VC);
                    qpsk_gl_fs_finish(theta, sw, VS, VC, &KF, &sn, &cs);
                } else if constexpr (TRIG) {
                    const qpsk_gl_split_arg g = qpsk_gl_split_prepare(theta, half, decltype(huge)::value);
                    const double rh = qpsk_gl_do_half(g.xa, g.dxa, half, tabh);
                    double DS, DC;
                    swap_halves(rh, &DS, &DC);
                    qpsk_gl_split_finish(theta, &g, DS, DC, &sn, &cs);
                }
                else if constexpr (decltype(huge)::value) qpsk_sincos_tab(theta, L.tab, L.tab_lo, &sn, &cs);
                else {
                    // the table row's loads first; under their LDS round trip the
                    // previous step's store, |theta| of its result (this step's
                    // argument) and the next symbol's read, then the polynomials
                    const qpsk_sincos_row row = qpsk_sincos_tab_load(theta, L.tab, L.tab_lo, &K);
                    __builtin_amdgcn_sched_barrier(0);
                    out[pend_k] = pend;
                    track();
                    __builtin_amdgcn_sched_barrier(0);
                    qpsk_sincos_tab_eval(&row, &K, &sn, &cs);
                }
                if constexpr (TRIG || decltype(huge)::value) {
                    // after the trig (the glibc pair issues its row's loads first)
                    out[pend_k] = pend;
                    track();
                }
                const d2 yn = widen(in[k + 1]);   // next symbol, read under this one's chain
                const double mi = y.x * cs + y.y * sn;
                const double mq = y.y * cs - y.x * sn;
                const float ri = static_cast<float>(mi), rq = static_cast<float>(mq);
                // e = +-1 (GetSign, :52-56): e*m is exact, so fma(ei, mq, -(eq*mi))
                // rounds the same exact difference as the reference's subtraction
                const bool qpos = rq >= 0.0f;
                const double ei = ri >= 0.0f ? 1.0 : -1.0;
                // eq*mi is mi or -mi exactly: a select of mi's sign (one
                // v_cndmask_b32 with a negated source, in place on the high
                // word) instead of a +-1.0 double (a select plus a copy of its
                // zero low word) and a multiply
                const double qmi = signsel(mi, qpos);
                const double pe = fma(ei, mq, -qmi);
                freq = freq + cb * pe;
                const double tn = theta + (freq + ca * pe);
                // single +-2pi wrap (:89-91) as a select: tn - copysign(2pi, tn)
                // is tn - 2pi above pi and tn + 2pi below -pi.  (sign(tn) *
                // (|tn| - 2pi) is one op shorter but gives -0 where the reference
                // gives +0, at tn = -2pi; fma(copysign(1, tn), -2pi, tn) is exact
                // too and measured 0.7 % slower at C2: tests/test_costas_identities.py,
                // profiles/r05_costas_wrap_forms_ab.txt)
                const double tw = tn - copysign(kTwoPi, tn);
                theta = fabs(tn) > kPi ? tw : tn;
                if constexpr (ROTB) {
                    // the decisions' sign bytes (byte 3 of the high words of +-1.0)
                    const uint32_t eih = static_cast<uint32_t>(__builtin_bit_cast(uint64_t, ei) >> 32);
                    const uint32_t eqh = qpos ? 0x3FF00000u : 0xBFF00000u;
                    pend = static_cast<uint16_t>(__builtin_amdgcn_perm(eqh, eih, 0x0c0c0703u));
                } else {
                    pend = f2{ri, rq};
                }
                pend_k = k;
                y = yn;
            };
            const double theta0 = theta, freq0 = freq;
            y = widen(in[0]);
            int k = 0;
            STAMP(tu);
            if (m >= mlo) {              // every stream the M&M ran uniformly
                // an even unroll: y and the next symbol alternate registers
                // instead of being copied back every symbol
                // by four (as the M&M loop): half the taken branches per symbol
                for (; k + 3 < mlo; k += 4) {   // uniform trip count
                    step(k, std::false_type{});
                    step(k + 1, std::false_type{});
                    step(k + 2, std::false_type{});
                    step(k + 3, std::false_type{});
                }
                if (k + 1 < mlo) {
                    step(k, std::false_type{});
                    step(k + 1, std::false_type{});
                    k += 2;
                }
                if (k < mlo) {
                    step(k, std::false_type{});
                    ++k;
                }
            }
            ACC(k_uni, tu);
#ifdef QPSK_LOOP_STAMPS
            k_uit += mlo;
#endif
            for (; k < m; ++k) step(k, std::false_type{});   // per-lane remainder (~1 symbol)
            out[pend_k] = pend;          // the round's last step
            track();
            // fmax drops NaN, which the fast path handles exactly like the full one
            // the fast pass's range: |theta| <= 2^40 (portable table), < 105414348
            // (glibc without __branred)
            const bool out_of_range = TRIG ? !(amax < QPSK_GLIBC_SMALL_LIMIT) && amax == amax : amax > 0x1p40;
            if (__builtin_expect(__ballot(cmine && out_of_range) != 0, 0)) {
                theta = theta0;
                freq = freq0;
                y = widen(in[0]);
                for (k = 0; k < m; ++k) step(k, std::true_type{});
                out[pend_k] = pend;
            }
            ACC(k_loop, tl);
        }
#ifdef QPSK_LOOP_STAMPS
        if (a.probe && lane == 0) {
            a.probe[blockIdx.x * 16 + 5] = k_bar;
            a.probe[blockIdx.x * 16 + 6] = k_loop;
            a.probe[blockIdx.x * 16 + 8] = k_uni;
            a.probe[blockIdx.x * 16 + 9] = k_uit;
        }
#endif
        if (real && mine) {
            a.state[s].theta = theta;
            a.state[s].freq = freq;
        }
        return;
    }

    // ================================================================ decode
    // the decode wave runs the real lanes only (its per-lane loop is off the chains)
    const bool dmine = real && mine;
    int diff_have = 0;
    float dpi = 0.f, dpq = 0.f;
    if (dmine) {
        diff_have = a.state[s].diff_have;
        dpi = a.state[s].diff_pi;
        dpq = a.state[s].diff_pq;
    }
    uint32_t *bits = (MODE == kModeDemodulate && dmine) ? a.bits + s * a.bits_stride_words : nullptr;
    f2 *syms = (SYMS && dmine) ? reinterpret_cast<f2 *>(a.syms) + s * a.syms_stride : nullptr;
    uint32_t word = 0;
    int wbits = 0;
    int64_t widx = 0, nbits = 0, ncs = 0;
    int err = 0;
    for (int r = 0; r <= NR + 1; ++r) {
        __builtin_amdgcn_s_barrier();
        if (r < 2) continue;
        const int slot = (r - 2) & 1;
        const int m = dmine ? L.cnt[((r - 2) & 3) * SPW + lane] : 0;
        const auto *in = L.rot + (slot * SPW + lane) * L.RS;
        for (int k = 0; k < m; ++k) {
            float ei, eq;
            if constexpr (ROTB) {
                const uint32_t db = in[k];
                ei = (db & 0x80u) ? -1.0f : 1.0f;
                eq = (db & 0x8000u) ? -1.0f : 1.0f;
            } else {
                const f2 rr = in[k];
                if (SYMS) {
                    if (ncs < a.syms_cap) syms[ncs] = rr;
                    else err |= 2;
                }
                // decision (QPSKDeModulator.cs:379-407)
                ei = rr.x >= 0.0f ? 1.0f : -1.0f;
                eq = rr.y >= 0.0f ? 1.0f : -1.0f;
            }
            ++ncs;
            if (MODE == kModeDemodulate) {
                // differential decode (QPSKDeModulator.cs:379-407, 304-337)
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
    if (!real) return;
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
    if (err) {
        atomicOr(&g->error, err);
        if (a.flags) atomicOr(a.flags, static_cast<uint32_t>(err));
    }
    if (a.n_bits) a.n_bits[s] = MODE == kModeDemodulate ? nbits : 0;
}

template <int SPW, int CAP, int KB, int TRIG, int ACT>
static int launch_loop_spw_t(const LoopArgs &a, const LoopParams &P, int mode, hipStream_t stream) {
    dim3 grid((a.S + SPW - 1) / SPW), block(256);
    const bool syms = a.syms != nullptr;
    const bool diff = P.differential != 0;
    if (mode == kModeConstellation)
        hipLaunchKernelGGL((loop_kernel<kModeConstellation, false, true, SPW, CAP, KB, TRIG, ACT>), grid, block, 0, stream, a, P);
    else if (diff && syms)
        hipLaunchKernelGGL((loop_kernel<kModeDemodulate, true, true, SPW, CAP, KB, TRIG, ACT>), grid, block, 0, stream, a, P);
    else if (diff)
        hipLaunchKernelGGL((loop_kernel<kModeDemodulate, true, false, SPW, CAP, KB, TRIG, ACT>), grid, block, 0, stream, a, P);
    else if (syms)
        hipLaunchKernelGGL((loop_kernel<kModeDemodulate, false, true, SPW, CAP, KB, TRIG, ACT>), grid, block, 0, stream, a, P);
    else
        hipLaunchKernelGGL((loop_kernel<kModeDemodulate, false, false, SPW, CAP, KB, TRIG, ACT>), grid, block, 0, stream, a, P);
    return static_cast<int>(grid.x);
}

template <int SPW, int CAP, int KB, int ACT = SPW>
static int launch_loop_spw(const LoopArgs &a, const LoopParams &P, int mode, hipStream_t stream) {
    return P.costas_trig ? launch_loop_spw_t<SPW, CAP, KB, 1, ACT>(a, P, mode, stream)
                         : launch_loop_spw_t<SPW, CAP, KB, 0, ACT>(a, P, mode, stream);
}

int launch_loop(const LoopArgs &a, const LoopParams &P, int mode, int variant, hipStream_t stream) {
    hipLaunchKernelGGL(carry_prefix_kernel, dim3(a.S), dim3(64), 0, stream, a);
    // The loop is latency-bound per stream; a wave's lanes are free, so the
    // default (sps >= 2) is 32 streams x 64-sample rounds.  Measured at C2
    // (profiles/archive/r01_loop_probe.txt): 16 x 64 and 16 x 128 (half the barriers)
    // both run slower per symbol.  sps < 2 needs the 80-symbol round capacity,
    // which fits LDS at 16 streams x 64.  variant (qpsk_demod_params.loop_variant)
    // forces 1 = 16 x 64, 2 = 32 x 64, 3 = 16 x 128; all compute identical results.
    if (P.sps < 2.0)
        return launch_loop_spw<16, kCapAny, 64>(a, P, mode, stream);
    else if (variant == 1)
        return launch_loop_spw<16, kCapSps2, 64>(a, P, mode, stream);
    else if (variant == 3)
        return launch_loop_spw<16, kCap128Sps2, 128>(a, P, mode, stream);
    else if (variant == 4 && P.sps >= 8.0)
        return launch_loop_spw<24, kCap128Sps8, 128>(a, P, mode, stream);
    else if (variant == 6 && P.sps >= 8.0)
        // 12 streams x 256-sample rounds, 32 busy lanes (20 shadow lanes on
        // row 0): a quarter of the rounds of 32 x 64, 135 KB of LDS
        return launch_loop_spw<12, kCap256Sps8, 256, 32>(a, P, mode, stream);
    else if (variant == 7 && P.sps >= 8.0)
        // 6 streams x 512-sample rounds, 26 shadow lanes: 137 KB of LDS
        return launch_loop_spw<6, kCap512Sps8, 512, 32>(a, P, mode, stream);
    else if (P.sps >= 8.0)
        return launch_loop_spw<32, kCapSps8, 64>(a, P, mode, stream);
    else if (P.sps >= 4.0)
        return launch_loop_spw<32, kCapSps4, 64>(a, P, mode, stream);
    else
        return launch_loop_spw<32, kCapSps2, 64>(a, P, mode, stream);
}

}  // namespace qpsk
