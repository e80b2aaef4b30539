// qpsk_kernels.h -- launch interface of the HIP kernels (qpsk_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "qpsk_state.h"

namespace qpsk {

constexpr int kModeDemodulate = 0;
constexpr int kModeConstellation = 1;

// Launch timestamps (qpsk_demod_enable_timing): kt[0] = the earliest
// workgroup start, kt[1] = the latest workgroup end of one kernel launch, in
// ticks of the 100 MHz wall clock (s_memrealtime; hipDeviceAttributeWallClockRate).
// The kernel's own span, as a kernel trace reports it, whichever streams its
// neighbours run on; recorded with vector atomics by a few lanes per launch.
__device__ __forceinline__ void kt_start(unsigned long long *kt) { atomicMin(kt, wall_clock64()); }
__device__ __forceinline__ void kt_end(unsigned long long *kt) { atomicMax(kt + 1, wall_clock64()); }
// Clock sample (timed calls): one thread's lifetime in shader-clock ticks
// (s_memtime) and wall ticks, added to clk[0], clk[1] when it goes out of
// scope; the ratio is the clock the kernel ran at (qpsk_demod_kernel_clocks)
struct ClkSample {
    unsigned long long *clk, c0, r0;
    __device__ explicit ClkSample(unsigned long long *p)
        : clk(p), c0(p ? __builtin_amdgcn_s_memtime() : 0), r0(p ? wall_clock64() : 0) {}
    __device__ ~ClkSample() {
        if (clk) {
            const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = wall_clock64();
            atomicAdd(clk, c1 - c0);
            atomicAdd(clk + 1, r1 - r0);
        }
    }
};
// records kt_end when it goes out of scope (every return path), lane 0 of each wave
struct KtEnd {
    unsigned long long *kt;
    __device__ ~KtEnd() {
        if (kt && (threadIdx.x & 63) == 0) kt_end(kt);
    }
};

// The CU a wave runs on, as an index < kCuKeys: XCC_ID, then HW_ID's SE, SH
// and CU fields (gfx9 layout: CU [11:8], SH [12], SE [15:13]).  Read from
// hardware registers (s_getreg); diagnostic use (FIR phases).
constexpr int kCuKeys = 2048;
__device__ __forceinline__ unsigned cu_key() {
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));     // hwreg(HW_REG_HW_ID)
    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));   // hwreg(HW_REG_XCC_ID)
    return ((((xcc & 7u) * 8u + ((hw >> 13) & 7u)) * 2u + ((hw >> 12) & 1u)) * 16u) + ((hw >> 8) & 15u);
}
// FIR phase sample (qpsk_demod_enable_fir_phases): phases[8 * shared + k],
// k = 0 stage (HBM -> LDS), 1 products and sums, 2 stores, 3 workgroups;
// shared = the loop kernel held the workgroup's CU when it started (cu_map)
constexpr int kFirPhaseWords = 16;

struct FirArgs {
    const float *x;        // [S][x_stride] float2 input
    int64_t x_stride;      // in float2
    const float *hist;     // [S][T-1] float2: previous call's last T-1 inputs
    const int64_t *lengths;
    int64_t n;             // uniform length when lengths == nullptr
    float *y;              // [S][y_stride] float2 output at y_offset
    int64_t y_stride;
    int64_t y_offset;
    unsigned long long *kt;   // launch timestamps or nullptr
    // or nullptr: {sum of shader-clock ticks, sum of wall ticks} over the
    // lifetimes of every kFirClockEvery-th workgroup (the clock the FIR runs at)
    unsigned long long *clk;
    // or nullptr: per-phase shader cycles of every kFirClockEvery-th workgroup,
    // split by whether a loop workgroup held its CU (cu_map, kCuKeys words)
    unsigned long long *phases;
    const unsigned *cu_map;
};
constexpr unsigned kFirClockEvery = 64;

struct LoopArgs {
    float *mf;             // [S][mf_stride] float2, MF output at kMfPrefix
    int64_t mf_stride;
    float *carry;          // [S][kCarryMax] float2
    const int64_t *lengths;
    int64_t n;
    StreamState *state;
    uint32_t *bits;        // [S][bits_stride_words]
    int64_t bits_stride_words;
    int64_t bits_cap_words;
    int64_t *n_bits;
    float *syms;           // [S][syms_stride] float2 or nullptr
    int64_t syms_stride;
    int64_t syms_cap;
    int64_t *n_syms;
    int S;
    unsigned long long *probe;   // diagnostic cycle stamps (QPSK_LOOP_STAMPS builds only)
    uint32_t *flags;       // per-handle OR of QPSK_STATUS_* raised by this call (or nullptr)
    int chunked;           // 1: an internal chunk of a longer call (StreamState.tofs runs on)
    unsigned long long *kt;   // launch timestamps or nullptr
    // residency counter (signal memory) or nullptr: every workgroup adds 1 as it
    // starts, so the next pipelined call's FIR can wait until the loop kernel
    // holds its CUs (qpsk_runtime.hip, process_async_one)
    unsigned long long *resident;
    unsigned long long *clk;   // clock sample of the M&M wave (ClkSample) or nullptr
    // or nullptr: cu_map[cu_key()] counts the workgroups of this launch that
    // hold that CU (FIR phase sample, FirArgs.phases)
    unsigned *cu_map;
};

// One internal chunk's rows appended behind what earlier chunks of the same
// call wrote: bits at per-stream bit offsets acc[s], symbols at acc[S + s]
// (first = the call's first chunk: offsets 0).
struct AppendArgs {
    uint8_t *dst_bits;           // [S][dst_bits_stride] or nullptr
    int64_t dst_bits_stride;     // bytes
    float *dst_syms;             // [S][dst_syms_stride] interleaved or nullptr
    int64_t dst_syms_stride;     // floats
    const uint32_t *src_bits;    // [S][src_bits_words] (MSB-first bytes)
    int64_t src_bits_words;
    const float *src_syms;       // [S][2 * src_syms_cap]
    int64_t src_syms_cap;
    const int64_t *counts;       // [2][S]: this chunk's n_bits, n_syms
    int64_t *acc;                // [2][S]: running totals
    int first;
    int last;                    // the call's last chunk: StreamState.tofs back to 0
    StreamState *state;
    int S;
};

struct FllArgs {
    const float *x;
    int64_t x_stride;
    float *y;
    int64_t y_stride;
    float *delay;          // [S][2*kFllTaps] float2
    const int64_t *lengths;
    int64_t n;
    StreamState *state;
    int S;
    unsigned long long *kt;   // launch timestamps or nullptr
    unsigned long long *clk;   // clock sample of each workgroup's first wave (ClkSample) or nullptr
};

struct IqbArgs {
    const float *x;        // [S][x_stride] float2
    int64_t x_stride;
    float *y;              // [S][y_stride] float2
    int64_t y_stride;
    const int64_t *lengths;
    int64_t n;
    StreamState *state;
    int S;
};

// Returns true when a specialised tile kernel was used.
// hrev_dev: the reversed RRC taps (ComplexFIRFilter._tapsIRev) in device memory.
bool launch_fir(const FirArgs &a, const float *hrev_dev, int T, int W, int S,
                int64_t n_max, hipStream_t stream);
void launch_fir_hist(const FirArgs &a, float *hist_new, int H, int S, hipStream_t stream);
// carry kernel + loop kernel; returns the loop kernel's workgroup count
int launch_loop(const LoopArgs &a, const LoopParams &P, int mode, int variant, hipStream_t stream);
void launch_append(const AppendArgs &a, hipStream_t stream);
void launch_iq_balance(const IqbArgs &a, hipStream_t stream);
void launch_fll(const FllArgs &a, const FllParams &P, hipStream_t stream);
void launch_fll_sys(const FllArgs &a, const FllParams &P, hipStream_t stream);   // qpsk_fll.hip

}  // namespace qpsk
