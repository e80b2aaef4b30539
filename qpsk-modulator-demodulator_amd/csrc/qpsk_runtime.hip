// qpsk_runtime.hip -- host runtime behind the C ABI (include/qpsk_demod.h):
// handle = a batch of S reference QPSKDeModulator instances living on one
// MI355X.  Owns the device buffers and the per-stream state, orders the kernels
// of one DeModulate call:
//
//     [FLL] -> matched-filter FIR -> FIR history carry -> M&M+Costas+decode
//
// qpsk_demod_process runs them on the handle's stream.  qpsk_demod_process_async
// splits each call into a front and a back stage on two library streams so
// that call k+1's front stage overlaps call k's back stage:
//
//     FLL off:  front = FIR + history        back = carry + loop kernel + copies
//     FLL on:   front = FLL                  back = FIR + history + carry + loop
//
// What the two stages share: the per-stream StreamState (its FLL fields are
// written only by the FLL, every other field only by the loop kernel), and the
// buffer at the stage boundary (MF rows, or FLL output rows), which is
// double-buffered (fll_out[2] / mf[2]; the second only when pipelined).
//
// Device layout (HBM, stream-major so every stage reads/writes each stream's
// time axis contiguously):
//   in      [S][n_max]              float2  staging for host input
//   fll_out [S][n_max]              float2  (FLL mode)
//   hist    2 x [S][T-1]            float2  FIR delay line (ping-pong)
//   mf      [2][S][256 + n_max]     float2  matched-filter output; the 256-slot
//                                           prefix receives the M&M carry (the
//                                           2nd only when pipelined)
//   carry   [S][256]                float2  M&M retained samples
//   state   [S]                     StreamState
//   bits    [S][words]              uint32  MSB-first packed bits
//   syms    [S][syms_cap]           float2  rotated symbols (on request)
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "qpsk_demod.h"
#include "qpsk_design.h"
#include "qpsk_kernels.h"

using namespace qpsk;

namespace {
thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

#define HIP_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return fail(QPSK_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <typename T>
int dev_alloc(T **p, size_t count) {
    *p = nullptr;
    if (count == 0) return QPSK_OK;
    hipError_t e = hipMalloc(reinterpret_cast<void **>(p), count * sizeof(T));
    if (e != hipSuccess)
        return fail(QPSK_ERR_DEVICE, std::string("hipMalloc: ") + hipGetErrorString(e));
    return QPSK_OK;
}

// launch-timestamp slots per timed call: FLL, FIR, loop kernel (start, end)
// and one spare pair; qpsk_demod_enable_timing records the first kKtCalls calls
constexpr int kKtPerCall = 12;   // spans: FLL 0-1, FIR 2-3, loop 4-5; clock sums: FIR 6-7, FLL 8-9, loop 10-11
constexpr int kKtCalls = 4096;
constexpr int64_t kMaxSamplesPerCall = int64_t(1) << 30;
// the symbol loop keeps sample indices of one call in 32-bit integers
constexpr int64_t kMaxCallSamples = (int64_t(1) << 31) - 129;
}  // namespace

namespace qpsk {
// shared error channel for the other C-ABI translation units (framer, synth)
int set_last_error(int code, const std::string &msg) { return fail(code, msg); }
}  // namespace qpsk

namespace {
struct Call {
    int32_t mode;
    const float *iq;
    int64_t stride_floats;
    int64_t n_samples;
    const int64_t *lengths;
    int32_t mem;
    uint8_t *bits;
    int64_t bits_stride_bytes;
    int64_t *n_bits;
    float *syms;
    int64_t syms_stride_floats;
    int64_t *n_syms;
    int64_t n_call = 0;    // derived by validate()
    int64_t max_sym = 0;
    // internal chunk of a longer call: outputs appended to dst_* at the running
    // offsets d_acc (first chunk: from 0), totals to n_bits / n_syms after the last
    bool append = false, first = false, last = false;
    uint8_t *dst_bits = nullptr;
    int64_t dst_bits_stride = 0;
    float *dst_syms = nullptr;
    int64_t dst_syms_stride = 0;
    int64_t *dst_n_bits = nullptr;   // device; written after the last chunk
    int64_t *dst_n_syms = nullptr;
};
}  // namespace

struct qpsk_demod {
    qpsk_demod_params p{};
    int S = 0;
    int T = 0;
    int W = 8;
    LoopDesign d;
    LoopParams lp{};
    int loop_variant = 0;
    FllParams fp{};
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int64_t n_max = 0;
    int64_t mf_stride = 0;       // float2
    int64_t bits_words = 0;      // per stream
    int64_t syms_cap = 0;        // per stream
    float *d_hrev = nullptr;
    float *d_in = nullptr;
    float *d_fll_out[2] = {nullptr, nullptr};
    float *d_iqb = nullptr;          // [S][n_max] float2, IQ_Balancer output (iq_balance only)
    float *d_hist[2] = {nullptr, nullptr};
    int hist_cur = 0;
    float *d_mf[2] = {nullptr, nullptr};
    float *d_carry = nullptr;
    StreamState *d_state = nullptr;
    float *d_fll_delay = nullptr;
    uint32_t *d_bits = nullptr;
    float *d_syms = nullptr;
    int64_t *d_counts = nullptr;     // [2][S]: n_bits, n_syms
    int64_t *d_lengths[2] = {nullptr, nullptr};
    int64_t *h_counts = nullptr;     // pinned
    // status flags (QPSK_STATUS_*): [0] = raised by device-memory calls since the
    // last qpsk_demod_status, [1] = raised by the current host-memory call
    uint32_t *d_flags = nullptr;
    uint32_t *h_flags = nullptr;     // pinned
    uint32_t status_host = 0;        // raised by host-memory calls since the last status
    // chunked calls (longer than max_samples_per_call): running per-stream
    // output offsets [2][S] and, for host-memory calls, device staging of the
    // whole call's output rows
    int64_t *d_acc = nullptr;
    uint8_t *d_xbits = nullptr;
    size_t xbits_bytes = 0;
    float *d_xsyms = nullptr;
    size_t xsyms_bytes = 0;
    bool timing = false;
    // launch timestamps of the timed calls ([call][kKtPerCall] wall-clock ticks,
    // written by the kernels themselves: qpsk_kernels.h kt_start / kt_end)
    unsigned long long *d_kt = nullptr;
    int kt_used = 0;
    // FIR phase sample (qpsk_demod_enable_fir_phases): per-phase cycle sums
    // [2][8] and the map of CUs a loop workgroup holds [kCuKeys]
    bool fir_phases = false;
    unsigned long long *d_phases = nullptr;
    unsigned *d_cu_map = nullptr;
    int wall_khz = 100000;
    int cus = 0;
    // ---- pipelined calls (qpsk_demod_process_async) ----------------------
    bool pipe_ready = false;
    int pipe_bufs = 0;               // 2 = double-buffered stage boundary, 1 = no room for it
    int pipe_cur = 0;
    hipStream_t s_front = nullptr, s_back = nullptr;
    hipEvent_t e_in = nullptr;
    hipEvent_t e_front[2] = {nullptr, nullptr}, e_back[2] = {nullptr, nullptr};
    bool front_rec[2] = {false, false}, back_rec[2] = {false, false};
    // FLL off: residency counter (signal memory) the loop kernel's workgroups
    // increment as they start; the next call's FIR waits for it to reach
    // resident_gate (see process_async_one)
    unsigned long long *d_resident = nullptr;
    uint64_t resident_issued = 0;    // workgroups of every gated loop launch so far
    uint64_t resident_gate = 0;      // what the newest gated loop launch brings it to, at least
    bool gate_pending = false;       // the next FIR has a loop launch to wait for
    // off under a profiler's counter collection (rocprofv3 --pmc serialises
    // every dispatch, so the wait would run to its cap on every call) or with
    // QPSK_PIPELINE_GATE=0
    bool use_gate = true;
    // the wait is bounded (gate_wait_kernel): at most gate_cap_ticks of the
    // wall clock (QPSK_GATE_TIMEOUT_MS, default 2000 ms), counted in d_gate[0]
    // when it runs out; gate_publish = false (QPSK_GATE_NO_PUBLISH=1 together
    // with QPSK_PIPELINE_GATE=1, tests only) keeps the loop workgroups from
    // counting, so every wait runs out
    unsigned *d_gate = nullptr;
    unsigned long long gate_cap_ticks = 0;
    bool gate_publish = true;
    int last_back = -1;              // boundary buffer of the newest back stage, -1 = none
    int64_t *h_len[2] = {nullptr, nullptr};   // pinned staging of per-call lengths
    // FLL on: the back stage (loop kernel) of the newest call is issued by the
    // next call, after that call's FLL, or by a flush (see process_async_one)
    hipEvent_t e_fll = nullptr;
    bool deferred = false;
    Call dcall{};
    int dbuf = 0;
    const int64_t *dlen = nullptr;
    unsigned long long *dkt = nullptr;
};

namespace qpsk {
// the pipelined path's front-stage stream (qpsk_rx.hip records "input consumed"
// on it); nullptr before the first pipelined call
hipStream_t pipe_front_stream(const qpsk_demod *h) { return h->s_front; }
int handle_streams(const qpsk_demod *h) { return h->S; }
int64_t handle_max_samples(const qpsk_demod *h) { return h->n_max; }
int handle_device(const qpsk_demod *h) { return h->p.device; }
int handle_sync(qpsk_demod *h);   // below: every queued call of the handle done
}  // namespace qpsk

namespace {

// The newest pipelined call's back stage, or nullptr.
hipEvent_t last_async(const qpsk_demod *h) { return h->last_back >= 0 ? h->e_back[h->last_back] : nullptr; }

int flush_deferred(qpsk_demod *h);   // issues a deferred back stage (with the stage runners)

// Host wait for every pipelined call issued so far (a deferred back stage is
// issued first: every caller of this waits for all of the handle's work).
int drain_async(qpsk_demod *h) {
    int rc;
    if ((rc = flush_deferred(h))) return rc;
    if (hipEvent_t e = last_async(h)) HIP_TRY(hipEventSynchronize(e));
    return QPSK_OK;
}


int validate(qpsk_demod *h, Call &c) {
    if (!h) return fail(QPSK_ERR_ARGUMENT_NULL, "null handle");
    if (c.mode != QPSK_MODE_DEMODULATE && c.mode != QPSK_MODE_CONSTELLATION)
        return fail(QPSK_ERR_ARGUMENT, "unknown mode");
    if (c.mem != QPSK_MEM_HOST && c.mem != QPSK_MEM_DEVICE) return fail(QPSK_ERR_ARGUMENT, "unknown mem");
    const int S = h->S;
    int64_t n_call = 0;
    if (c.lengths) {
        for (int s = 0; s < S; ++s) {
            if (c.lengths[s] < 0) return fail(QPSK_ERR_ARGUMENT, "negative length");
            n_call = std::max(n_call, c.lengths[s]);
        }
    } else {
        if (c.n_samples < 0) return fail(QPSK_ERR_ARGUMENT, "negative n_samples");
        n_call = c.n_samples;
    }
    if (n_call > kMaxCallSamples)
        return fail(QPSK_ERR_OUT_OF_RANGE, "calls above 2^31 - 129 samples per stream (a C# span holds 2^30)");
    if (n_call > 0 && !c.iq) return fail(QPSK_ERR_ARGUMENT_NULL, "SamplesIQ is null");
    if (n_call > 0 && c.stride_floats < 2 * n_call) return fail(QPSK_ERR_ARGUMENT, "stride too small");
    if (c.mode == QPSK_MODE_DEMODULATE && (!c.bits || !c.n_bits))
        return fail(QPSK_ERR_ARGUMENT_NULL, "bits / n_bits required");
    if (c.mode == QPSK_MODE_CONSTELLATION && (!c.syms || !c.n_syms))
        return fail(QPSK_ERR_ARGUMENT_NULL, "syms / n_syms required");
    const int64_t max_sym = qpsk_demod_max_symbols(h, n_call);
    if (c.bits && c.bits_stride_bytes < ((2 * max_sym + 7) / 8))
        return fail(QPSK_ERR_ARGUMENT, "bits_stride_bytes smaller than 2*max_symbols/8");
    if (c.syms && c.syms_stride_floats < 2 * max_sym)
        return fail(QPSK_ERR_ARGUMENT, "syms_stride_floats smaller than 2*max_symbols");
    if (n_call > 0 && c.mem == QPSK_MEM_DEVICE && (c.stride_floats & 1))
        return fail(QPSK_ERR_ARGUMENT, "device stride_floats must be even");
    int rc;
    if (c.syms && !h->d_syms) {
        // on the handle's device whatever the calling thread's current one is
        // (a group's worker threads, qpsk_group.cpp)
        HIP_TRY(hipSetDevice(h->p.device));
        if ((rc = dev_alloc(&h->d_syms, static_cast<size_t>(2 * S * h->syms_cap)))) return rc;
    }
    c.n_call = n_call;
    c.max_sym = max_sym;
    return QPSK_OK;
}

// the launch-timestamp slots of the next timed call, or nullptr
unsigned long long *next_kt(qpsk_demod *h) {
    if (!h->timing || !h->d_kt || h->kt_used >= kKtCalls) return nullptr;
    return h->d_kt + static_cast<size_t>(kKtPerCall) * h->kt_used++;
}

}  // namespace (validation)

namespace {

// optional IQ_Balancer pre-stage (IQ Balancer.cs:15-25) into d_iqb
void run_iqb(qpsk_demod *h, const float *x, int64_t x_stride, const int64_t *d_len, int64_t n_call,
             hipStream_t st) {
    IqbArgs ia{};
    ia.x = x; ia.x_stride = x_stride;
    ia.y = h->d_iqb; ia.y_stride = h->n_max;
    ia.lengths = d_len; ia.n = n_call;
    ia.state = h->d_state; ia.S = h->S;
    launch_iq_balance(ia, st);
}

// FLL (Band-Edge Filter.cs:64-87), README order FLL -> MF
void run_fll(qpsk_demod *h, const float *x, int64_t x_stride, const int64_t *d_len, int64_t n_call,
             float *y, hipStream_t st, unsigned long long *kt) {
    FllArgs fa{};
    fa.x = x; fa.x_stride = x_stride;
    fa.y = y; fa.y_stride = h->n_max;
    fa.delay = h->d_fll_delay;
    fa.lengths = d_len; fa.n = n_call;
    fa.state = h->d_state; fa.S = h->S;
    fa.kt = kt ? kt + 0 : nullptr;
    fa.clk = kt ? kt + 8 : nullptr;
    launch_fll(fa, h->fp, st);
}

// matched filter (QPSKDeModulator.cs:360) + FIR delay-line carry
int run_fir(qpsk_demod *h, const float *x, int64_t x_stride, const int64_t *d_len, int64_t n_call,
            float *mf, hipStream_t st, unsigned long long *kt) {
    FirArgs fa{};
    fa.x = x; fa.x_stride = x_stride;
    fa.hist = h->d_hist[h->hist_cur];
    fa.lengths = d_len; fa.n = n_call;
    fa.y = mf; fa.y_stride = h->mf_stride; fa.y_offset = kMfPrefix;
    fa.kt = kt ? kt + 2 : nullptr;
    fa.clk = kt ? kt + 6 : nullptr;
    if (h->fir_phases) {
        fa.phases = h->d_phases;
        fa.cu_map = h->d_cu_map;
    }
    if (n_call > 0) {
        launch_fir(fa, h->d_hrev, h->T, h->W, h->S, n_call, st);
        fa.kt = nullptr;
        fa.clk = nullptr;
        fa.phases = nullptr;
        launch_fir_hist(fa, h->d_hist[h->hist_cur ^ 1], h->T - 1, h->S, st);
        h->hist_cur ^= 1;
    }
    return QPSK_OK;
}

// The residency gate of the pipelined path (process_async_one): one wave on
// the front stream, ahead of the FIR, polls the counter the loop kernel's
// workgroups bump as they start (s_sleep between reads) and ends when it
// reaches target -- or when cap wall-clock ticks have passed, counted in
// *timeouts.  The FIR behind it in stream order is dispatched only then, as
// with hipStreamWaitValue64, but a counter that never arrives (a dispatch
// serialised by a tool the environment predicate does not know) costs one cap
// per call instead of a hang.  The gate orders dispatch only; no result
// depends on it.
__global__ void gate_wait_kernel(const unsigned long long *resident, unsigned long long target,
                                 unsigned long long cap, unsigned *timeouts) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(resident, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
        if (wall_clock64() - t0 > cap) {
            atomicAdd(timeouts, 1u);
            return;
        }
        __builtin_amdgcn_s_sleep(4);
    }
}

int gate_wait(qpsk_demod *h, hipStream_t st) {
    if (!h->gate_pending) return QPSK_OK;
    h->gate_pending = false;
    hipLaunchKernelGGL(gate_wait_kernel, dim3(1), dim3(64), 0, st, h->d_resident,
                       static_cast<unsigned long long>(h->resident_gate), h->gate_cap_ticks, h->d_gate);
    HIP_TRY(hipGetLastError());
    return QPSK_OK;
}

// symbol sync + Costas + decode (QPSKDeModulator.cs:364-408) and the output copies
// resident: the pipelined path's residency counter (nullptr otherwise); the
// launch's workgroup count is added to h->resident_issued
int run_loop(qpsk_demod *h, const Call &c, const int64_t *d_len, float *mf, hipStream_t st,
             unsigned long long *kt, unsigned long long *resident = nullptr) {
    const int S = h->S;
    LoopArgs la{};
    la.mf = mf; la.mf_stride = h->mf_stride;
    la.carry = h->d_carry;
    la.lengths = d_len; la.n = c.n_call;
    la.state = h->d_state;
    la.bits = c.mode == QPSK_MODE_DEMODULATE ? h->d_bits : nullptr;
    la.bits_stride_words = h->bits_words;
    la.bits_cap_words = h->bits_words;
    la.n_bits = h->d_counts;
    la.syms = c.syms ? h->d_syms : nullptr;
    la.syms_stride = h->syms_cap;
    la.syms_cap = h->syms_cap;
    la.n_syms = h->d_counts + S;
    // device-memory outputs whose rows the kernel can address as its own (4-B
    // aligned word rows holding every word a row can take; float2-aligned
    // symbol rows): written in place, no staging copy behind the kernel
    const int64_t need_words = (2 * c.max_sym + 31) / 32;
    const bool direct_bits = !c.append && c.mem == QPSK_MEM_DEVICE && la.bits && c.n_bits &&
                             (reinterpret_cast<uintptr_t>(c.n_bits) & 7) == 0 &&
                             (reinterpret_cast<uintptr_t>(c.bits) & 3) == 0 && (c.bits_stride_bytes & 3) == 0 &&
                             c.bits_stride_bytes / 4 >= need_words;
    const bool direct_syms = !c.append && c.mem == QPSK_MEM_DEVICE && c.syms &&
                             (reinterpret_cast<uintptr_t>(c.syms) & 7) == 0 && (c.syms_stride_floats & 1) == 0 &&
                             c.syms_stride_floats / 2 >= c.max_sym;
    if (direct_bits) {
        la.bits = reinterpret_cast<uint32_t *>(c.bits);
        la.bits_stride_words = c.bits_stride_bytes / 4;
        la.bits_cap_words = c.bits_stride_bytes / 4;
        la.n_bits = c.n_bits;
    }
    if (direct_syms) {
        la.syms = c.syms;
        la.syms_stride = c.syms_stride_floats / 2;
        la.syms_cap = c.syms_stride_floats / 2;
        if (c.n_syms && (reinterpret_cast<uintptr_t>(c.n_syms) & 7) == 0) la.n_syms = c.n_syms;
    }
    la.S = S;
    // host-memory calls (chunks of one included) raise into slot 1, which the
    // call clears first and reads back at its end; device-memory calls into
    // slot 0, read by qpsk_demod_status
    la.flags = h->d_flags + (c.mem == QPSK_MEM_HOST ? 1 : 0);
    la.chunked = c.append ? 1 : 0;
    la.kt = kt ? kt + 4 : nullptr;
    la.clk = kt ? kt + 10 : nullptr;
    la.cu_map = h->fir_phases ? h->d_cu_map : nullptr;
    la.resident = h->gate_publish ? resident : nullptr;
    const int grid = launch_loop(la, h->lp, c.mode, h->loop_variant, st);
    HIP_TRY(hipGetLastError());
    if (resident) {
        // the next FIR may start once min(grid, CUs) workgroups hold their CUs:
        // at most one 104-147 KB loop workgroup fits a CU, and those are the
        // first ones dispatched (never more than there are)
        h->resident_gate = h->resident_issued + static_cast<uint64_t>(std::min(grid, std::max(h->cus, 1)));
        h->resident_issued += static_cast<uint64_t>(grid);
        h->gate_pending = true;
    }
    if (c.append) {
        AppendArgs aa{};
        aa.dst_bits = c.mode == QPSK_MODE_DEMODULATE ? c.dst_bits : nullptr;
        aa.dst_bits_stride = c.dst_bits_stride;
        aa.dst_syms = c.syms ? c.dst_syms : nullptr;
        aa.dst_syms_stride = c.dst_syms_stride;
        aa.src_bits = h->d_bits;
        aa.src_bits_words = h->bits_words;
        aa.src_syms = h->d_syms;
        aa.src_syms_cap = h->syms_cap;
        aa.counts = h->d_counts;
        aa.acc = h->d_acc;
        aa.first = c.first ? 1 : 0;
        aa.last = c.last ? 1 : 0;
        aa.state = h->d_state;
        aa.S = S;
        launch_append(aa, st);
        HIP_TRY(hipGetLastError());
        if (c.last) {
            if (c.dst_n_bits)
                HIP_TRY(hipMemcpyAsync(c.dst_n_bits, h->d_acc, S * sizeof(int64_t), hipMemcpyDeviceToDevice, st));
            if (c.dst_n_syms)
                HIP_TRY(hipMemcpyAsync(c.dst_n_syms, h->d_acc + S, S * sizeof(int64_t), hipMemcpyDeviceToDevice, st));
        }
        return QPSK_OK;
    }
    const hipMemcpyKind kind = c.mem == QPSK_MEM_HOST ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    const int64_t bytes_row = (2 * c.max_sym + 7) / 8;
    if (c.bits && bytes_row > 0 && !direct_bits)
        HIP_TRY(hipMemcpy2DAsync(c.bits, c.bits_stride_bytes, h->d_bits, h->bits_words * 4, bytes_row, S, kind, st));
    if (c.syms && c.max_sym > 0 && !direct_syms)
        HIP_TRY(hipMemcpy2DAsync(c.syms, c.syms_stride_floats * sizeof(float), h->d_syms,
                                 2 * h->syms_cap * sizeof(float), 2 * c.max_sym * sizeof(float), S, kind, st));
    if (c.mem == QPSK_MEM_HOST) {
        HIP_TRY(hipMemcpyAsync(h->h_counts, h->d_counts, 2 * S * sizeof(int64_t), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(h->h_flags, h->d_flags + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (c.n_bits) std::memcpy(c.n_bits, h->h_counts, S * sizeof(int64_t));
        if (c.n_syms) std::memcpy(c.n_syms, h->h_counts + S, S * sizeof(int64_t));
        h->status_host |= *h->h_flags;
    } else {
        if (c.n_bits && !direct_bits) HIP_TRY(hipMemcpyAsync(c.n_bits, h->d_counts, S * sizeof(int64_t), kind, st));
        if (c.n_syms && !(direct_syms && la.n_syms == c.n_syms))
            HIP_TRY(hipMemcpyAsync(c.n_syms, h->d_counts + S, S * sizeof(int64_t), kind, st));
    }
    return QPSK_OK;
}

}  // namespace (stage runners)

namespace {

// Streams, events and the second stage-boundary buffer of the pipelined path.
// The back stream gets the device's highest priority: its loop kernel is the
// latency-bound stage, the front stage fills the CUs it leaves idle.
int pipe_setup(qpsk_demod *h) {
    if (h->pipe_ready) return QPSK_OK;
    // every step is guarded: a set-up that failed part way runs again on the
    // next pipelined call and completes what is missing, leaking nothing and
    // keeping (not re-zeroing) the counters it already made
    int least = 0, greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
    if (!h->s_front) HIP_TRY(hipStreamCreateWithPriority(&h->s_front, hipStreamNonBlocking, least));
    if (!h->s_back) HIP_TRY(hipStreamCreateWithPriority(&h->s_back, hipStreamNonBlocking, greatest));
    if (!h->e_in) HIP_TRY(hipEventCreateWithFlags(&h->e_in, hipEventDisableTiming));
    for (int b = 0; b < 2; ++b) {
        if (!h->e_front[b]) HIP_TRY(hipEventCreateWithFlags(&h->e_front[b], hipEventDisableTiming));
        if (!h->e_back[b]) HIP_TRY(hipEventCreateWithFlags(&h->e_back[b], hipEventDisableTiming));
        if (!h->h_len[b]) HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&h->h_len[b]), h->S * sizeof(int64_t)));
    }
    if (!h->e_fll) HIP_TRY(hipEventCreateWithFlags(&h->e_fll, hipEventDisableTiming));
    if (!h->d_resident) {
        HIP_TRY(hipExtMallocWithFlags(reinterpret_cast<void **>(&h->d_resident), sizeof(unsigned long long),
                                      hipMallocSignalMemory));
        HIP_TRY(hipMemset(h->d_resident, 0, sizeof(unsigned long long)));
    }
    int rc;
    if (!h->d_gate) {
        if ((rc = dev_alloc(&h->d_gate, 1))) return rc;
        HIP_TRY(hipMemset(h->d_gate, 0, sizeof(unsigned)));
    }
    if (!h->d_lengths[1] && (rc = dev_alloc(&h->d_lengths[1], h->S))) return rc;
    // the second boundary buffer: MF rows (the FIR of one call writes one while
    // the loop kernel of the previous call reads the other).  No room for it
    // (batches near the 288 GB) -> calls still queue back to back, but each
    // front stage waits for the previous back stage
    const size_t S = static_cast<size_t>(h->S);
    if (!h->d_mf[1]) {
        hipError_t e = hipMalloc(reinterpret_cast<void **>(&h->d_mf[1]), 2 * S * h->mf_stride * sizeof(float));
        if (e != hipSuccess) {
            (void)hipGetLastError();
            h->d_mf[1] = nullptr;
        } else {
            HIP_TRY(hipMemset(h->d_mf[1], 0, 2 * S * h->mf_stride * sizeof(float)));
        }
    }
    h->pipe_bufs = h->d_mf[1] ? 2 : 1;
    h->pipe_ready = true;
    return QPSK_OK;
}

}  // namespace (pipeline setup)

extern "C" {

int qpsk_abi_version(void) { return QPSK_ABI_VERSION; }

const char *qpsk_last_error(void) { return g_last_error.c_str(); }

void qpsk_demod_params_init(qpsk_demod_params *p, int32_t sample_rate, int32_t symbol_rate) {
    std::memset(p, 0, sizeof(*p));
    p->sample_rate = sample_rate;
    p->symbol_rate = symbol_rate;
    p->rrc_alpha = 0.9f;                       // QPSKDeModulator.cs:14-18 defaults
    p->rrc_span = 6;
    p->symbol_sync_bandwidth = 0.0001;
    p->costas_loop_bandwidth = 120;
    p->cfo_loop_bandwidth = static_cast<double>(0.0001f);
    p->differential = 1;
    p->enable_fll = 0;
    p->vector_lanes = 8;
    p->device = 0;
    p->max_samples_per_call = 1 << 20;
}

int64_t qpsk_demod_max_symbols(const qpsk_demod *h, int64_t n) {
    if (!h || n <= 0) return 0;
    // every symbol but the first advances the M&M clock by >= sps - 0.1 samples
    const double min_adv = h->lp.sps - 0.1;
    int64_t bound = n;
    if (min_adv > 0.5) {
        const double b = std::ceil(static_cast<double>(n + kCarryMax) / min_adv) + 4.0;
        if (b < static_cast<double>(n)) bound = static_cast<int64_t>(b);
    }
    return bound;
}

int qpsk_demod_create(const qpsk_demod_params *p, int32_t n_streams, qpsk_demod **out) {
    if (!p || !out) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    *out = nullptr;
    if (n_streams <= 0) return fail(QPSK_ERR_ARGUMENT, "n_streams must be positive");
    if (p->max_samples_per_call <= 0) return fail(QPSK_ERR_ARGUMENT, "max_samples_per_call must be positive");
    // the symbol loop counts a chunk's samples in 32-bit integers; a longer
    // call is split into chunks of max_samples_per_call (a C# span holds at
    // most 2^31 - 1 floats anyway)
    if (p->max_samples_per_call > kMaxSamplesPerCall)
        return fail(QPSK_ERR_OUT_OF_RANGE, "max_samples_per_call above 2^30");
    auto *h = new qpsk_demod();
    h->p = *p;
    h->S = n_streams;
    h->W = p->vector_lanes <= 1 ? 1 : p->vector_lanes;
    if (h->W != 1 && h->W != 4 && h->W != 8 && h->W != 16) {
        delete h;
        return fail(QPSK_ERR_ARGUMENT, "vector_lanes must be 1, 4, 8 or 16");
    }
    if (p->loop_variant < 0 || p->loop_variant > 7) {
        delete h;
        return fail(QPSK_ERR_ARGUMENT, "loop_variant must be 0..7");
    }
    std::string err;
    int rc = design_loops(p->sample_rate, p->symbol_rate, p->rrc_alpha, p->rrc_span,
                          p->symbol_sync_bandwidth, p->costas_loop_bandwidth, p->cfo_loop_bandwidth,
                          &h->d, &err);
    if (rc != QPSK_OK) {
        delete h;
        return fail(rc, err);
    }
    h->T = static_cast<int>(h->d.rrc_f32.size());
    h->lp.sps = h->d.mm_sps;
    h->lp.kp = h->d.kp;
    h->lp.ki = h->d.ki;
    h->lp.c_alpha = h->d.costas_alpha;
    h->lp.c_beta = h->d.costas_beta;
    h->lp.differential = p->differential ? 1 : 0;
    if (p->costas_trig != 0 && p->costas_trig != 1) {
        delete h;
        return fail(QPSK_ERR_ARGUMENT, "costas_trig must be 0 (portable) or 1 (glibc)");
    }
    h->lp.costas_trig = p->costas_trig;
    h->loop_variant = p->loop_variant;
    h->fp.beta = h->d.fll_beta;
    h->fp.alpha = h->d.fll_alpha;
    h->fp.max_freq = h->d.fll_max_freq;
    h->fp.min_freq = -h->d.fll_max_freq;
    h->fp.lanes = h->W;
    for (int k = 0; k < kFllTaps; ++k) {
        const int src = kFllTaps - 1 - k;
        h->fp.lower_rev[2 * k] = h->d.fll_lower_iq[2 * src];
        h->fp.lower_rev[2 * k + 1] = h->d.fll_lower_iq[2 * src + 1];
        h->fp.upper_rev[2 * k] = h->d.fll_upper_iq[2 * src];
        h->fp.upper_rev[2 * k + 1] = h->d.fll_upper_iq[2 * src + 1];
    }
    // the systolic FLL shares the products of both band-edge filters, which needs
    // upper = conj(lower) exactly (Band-Edge Filter.cs:176-178 builds it so)
    h->fp.conj_taps = 1;
    for (int k = 0; k < 2 * kFllTaps; ++k) {
        uint32_t lo, up;
        std::memcpy(&lo, &h->fp.lower_rev[k], 4);
        std::memcpy(&up, &h->fp.upper_rev[k], 4);
        if (up != ((k & 1) ? (lo ^ 0x80000000u) : lo)) h->fp.conj_taps = 0;
    }

    auto cleanup_fail = [&](int code) {
        qpsk_demod_destroy(h);
        return code;
    };
    if (hipSetDevice(p->device) != hipSuccess)
        return cleanup_fail(fail(QPSK_ERR_DEVICE, "hipSetDevice failed (no GPU?)"));
    // auto loop shape at sps >= 8: 24 streams x 128-sample rounds halve the
    // per-round bookkeeping per symbol (C2 loop 23.9 -> 22.2-22.95 ms, A/B x3 on
    // one MI355X) but take 147 KB of LDS, one workgroup per CU; above one
    // workgroup per CU (C5: 8192 streams = 342 workgroups) the 32 x 64 shape
    // (256 workgroups) is the faster one (C5 serial loop 24.0 vs 39.2 ms).
    // Above half the CUs, too: no FIR workgroup fits beside a 147 KB one, and
    // pipelined calls then wait for the FIR (4096 streams: 37.7 vs 33.4 ms a
    // call; 2048: 24.6 vs 29.1 ms, profiles/archive/r02_loop_shapes_c4_ab.txt)
    if (hipDeviceGetAttribute(&h->cus, hipDeviceAttributeMultiprocessorCount, p->device) != hipSuccess)
        h->cus = 0;
    if (hipDeviceGetAttribute(&h->wall_khz, hipDeviceAttributeWallClockRate, p->device) != hipSuccess ||
        h->wall_khz <= 0)
        h->wall_khz = 100000;
    // Round 4: long rounds with shadow lanes (6 x 512, 12 x 256: 32 busy lanes,
    // a quarter / half of the per-round bookkeeping per symbol of 24 x 128)
    // beat it wherever they fit the chip in one pass, at sps >= 8, A/B on one
    // MI355X (profiles/r04_loop_long_rounds_ab.txt): 256 streams 13.6 -> 14.4
    // GSa/s (C2), 1024: 48.5 / 51.2 / 54.5 (24 x 128 / 12 x 256 / 6 x 512),
    // 2048: 88.4 / 99.3 (32 x 64: 74.6).  Above 12 x 256's one pass (4096
    // streams, C4) the 32 x 64 default stays: more workgroups than CUs, and
    // half-empty waves cost the FIR beside them issue slots
    h->loop_variant = qpsk_demod_pick_loop_variant(h->loop_variant, h->S, h->lp.sps, h->cus);
    h->use_gate = qpsk_pipeline_gate_enabled() == 1;
    {
        const char *v = std::getenv("QPSK_GATE_TIMEOUT_MS");
        const long ms = v && *v ? std::strtol(v, nullptr, 10) : 2000;
        h->gate_cap_ticks = static_cast<unsigned long long>(ms > 0 ? ms : 1) * static_cast<unsigned>(h->wall_khz);
        // test hook, honoured only beside an explicit QPSK_PIPELINE_GATE=1: a
        // stray QPSK_GATE_NO_PUBLISH alone must not make every call wait out the cap
        const char *np = std::getenv("QPSK_GATE_NO_PUBLISH");
        const char *force = std::getenv("QPSK_PIPELINE_GATE");
        const bool forced = force && std::strcmp(force, "1") == 0;
        h->gate_publish = !(forced && np && *np && std::strcmp(np, "0") != 0);
    }
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
        return cleanup_fail(fail(QPSK_ERR_DEVICE, "hipStreamCreate failed"));
    h->own_stream = true;

    const int64_t S = n_streams;
    h->n_max = p->max_samples_per_call;
    h->mf_stride = ((kMfPrefix + h->n_max + 2 + 63) / 64) * 64;   // + row slack for the loop loader
    h->syms_cap = qpsk_demod_max_symbols(h, h->n_max);
    h->bits_words = (2 * h->syms_cap + 31) / 32 + 1;
    const int H = h->T - 1;
    if ((rc = dev_alloc(&h->d_hrev, h->T)) || (rc = dev_alloc(&h->d_hist[0], 2 * S * H)) ||
        (rc = dev_alloc(&h->d_hist[1], 2 * S * H)) ||
        (rc = dev_alloc(&h->d_mf[0], static_cast<size_t>(2 * S * h->mf_stride))) ||
        (rc = dev_alloc(&h->d_carry, 2 * S * kCarryMax)) || (rc = dev_alloc(&h->d_state, S)) ||
        (rc = dev_alloc(&h->d_fll_delay, 2 * S * 2 * kFllTaps)) ||
        (rc = dev_alloc(&h->d_bits, static_cast<size_t>(S * h->bits_words))) ||
        (rc = dev_alloc(&h->d_counts, 2 * S)) || (rc = dev_alloc(&h->d_lengths[0], S)))
        return cleanup_fail(rc);
    if (p->enable_fll && (rc = dev_alloc(&h->d_fll_out[0], static_cast<size_t>(2 * S * h->n_max))))
        return cleanup_fail(rc);
    if (p->iq_balance && (rc = dev_alloc(&h->d_iqb, static_cast<size_t>(2 * S * h->n_max))))
        return cleanup_fail(rc);
    if (hipHostMalloc(reinterpret_cast<void **>(&h->h_counts), 2 * S * sizeof(int64_t)) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void **>(&h->h_flags), sizeof(uint32_t)) != hipSuccess)
        return cleanup_fail(fail(QPSK_ERR_DEVICE, "hipHostMalloc"));
    if ((rc = dev_alloc(&h->d_flags, 2)) || hipMemset(h->d_flags, 0, 2 * sizeof(uint32_t)) != hipSuccess)
        return cleanup_fail(rc ? rc : fail(QPSK_ERR_DEVICE, "hipMemset"));
    std::vector<float> hrev(h->T);
    for (int k = 0; k < h->T; ++k) hrev[k] = h->d.rrc_f32[h->T - 1 - k];
    // Fresh instances: zero delay lines (FIRFilter.cs:50-51), M&M baseIndex = 1
    // (MuellerMuller.cs:44), everything else zero.
    std::vector<StreamState> st(S);
    for (auto &x : st) {
        std::memset(&x, 0, sizeof(x));
        x.base = 1;
    }
    if (hipMemcpy(h->d_hrev, hrev.data(), h->T * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(h->d_state, st.data(), S * sizeof(StreamState), hipMemcpyHostToDevice) != hipSuccess ||
        (H > 0 && hipMemset(h->d_hist[0], 0, 2 * S * H * sizeof(float)) != hipSuccess) ||
        hipMemset(h->d_carry, 0, 2 * S * kCarryMax * sizeof(float)) != hipSuccess ||
        hipMemset(h->d_fll_delay, 0, 2 * S * 2 * kFllTaps * sizeof(float)) != hipSuccess ||
        hipMemset(h->d_mf[0], 0, static_cast<size_t>(2 * S * h->mf_stride) * sizeof(float)) != hipSuccess)
        return cleanup_fail(fail(QPSK_ERR_DEVICE, "device init failed"));
    *out = h;
    return QPSK_OK;
}

int qpsk_demod_destroy(qpsk_demod *h) {
    if (!h) return QPSK_OK;
    (void)hipSetDevice(h->p.device);   // frees and stream teardown on the handle's device
    drain_async(h);
    if (h->stream) hipStreamSynchronize(h->stream);
    hipFree(h->d_hrev);
    hipFree(h->d_in);
    for (int b = 0; b < 2; ++b) {
        hipFree(h->d_fll_out[b]);
        hipFree(h->d_hist[b]);
        hipFree(h->d_mf[b]);
        hipFree(h->d_lengths[b]);
        if (h->h_len[b]) hipHostFree(h->h_len[b]);
        if (h->e_front[b]) hipEventDestroy(h->e_front[b]);
        if (h->e_back[b]) hipEventDestroy(h->e_back[b]);
    }
    if (h->d_resident) hipFree(h->d_resident);
    hipFree(h->d_gate);
    hipFree(h->d_kt);
    hipFree(h->d_phases);
    hipFree(h->d_cu_map);
    hipFree(h->d_carry);
    hipFree(h->d_iqb);
    hipFree(h->d_state);
    hipFree(h->d_fll_delay);
    hipFree(h->d_bits);
    hipFree(h->d_syms);
    hipFree(h->d_counts);
    if (h->h_counts) hipHostFree(h->h_counts);
    if (h->h_flags) hipHostFree(h->h_flags);
    hipFree(h->d_flags);
    hipFree(h->d_acc);
    hipFree(h->d_xbits);
    hipFree(h->d_xsyms);
    if (h->e_in) hipEventDestroy(h->e_in);
    if (h->e_fll) hipEventDestroy(h->e_fll);
    if (h->s_front) hipStreamDestroy(h->s_front);
    if (h->s_back) hipStreamDestroy(h->s_back);
    if (h->own_stream && h->stream) hipStreamDestroy(h->stream);
    delete h;
    return QPSK_OK;
}

int qpsk_demod_set_stream(qpsk_demod *h, void *hip_stream) {
    if (!h) return fail(QPSK_ERR_ARGUMENT_NULL, "null handle");
    HIP_TRY(hipSetDevice(h->p.device));
    int rc;
    if ((rc = drain_async(h))) return rc;
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (hip_stream) {
        if (h->own_stream) hipStreamDestroy(h->stream);
        h->stream = static_cast<hipStream_t>(hip_stream);
        h->own_stream = false;
    } else if (!h->own_stream) {
        HIP_TRY(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
        h->own_stream = true;
    }
    return QPSK_OK;
}

int qpsk_demod_enable_timing(qpsk_demod *h, int32_t on) {
    if (!h) return fail(QPSK_ERR_ARGUMENT_NULL, "null handle");
    h->kt_used = 0;
    h->timing = on != 0;
    if (!h->timing) return QPSK_OK;
    HIP_TRY(hipSetDevice(h->p.device));
    int rc;
    const size_t n = static_cast<size_t>(kKtCalls) * kKtPerCall;
    if (!h->d_kt && (rc = dev_alloc(&h->d_kt, n))) return rc;
    // (start, end) pairs of slots 0-5: start = +inf for the atomic minimum, end
    // = 0 for the maximum; slots 6-11 (clock sums) = 0
    std::vector<unsigned long long> init(n, 0ull);
    for (size_t i = 0; i < n; i += 2)
        if (i % kKtPerCall < 6) init[i] = ~0ull;
    if ((rc = drain_async(h))) return rc;
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipMemcpy(h->d_kt, init.data(), n * sizeof(unsigned long long), hipMemcpyHostToDevice));
    return QPSK_OK;
}

int qpsk_demod_enable_fir_phases(qpsk_demod *h, int32_t on) {
    if (!h) return fail(QPSK_ERR_ARGUMENT_NULL, "null handle");
    int rc;
    if ((rc = drain_async(h))) return rc;
    HIP_TRY(hipSetDevice(h->p.device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (on && (!h->d_phases || !h->d_cu_map)) {
        // both or neither: a half-allocated pair would let the sampled FIR
        // workgroups read a null cu_map
        if ((!h->d_phases && (rc = dev_alloc(&h->d_phases, kFirPhaseWords))) ||
            (!h->d_cu_map && (rc = dev_alloc(&h->d_cu_map, kCuKeys)))) {
            hipFree(h->d_phases);
            hipFree(h->d_cu_map);
            h->d_phases = nullptr;
            h->d_cu_map = nullptr;
            return rc;
        }
        HIP_TRY(hipMemset(h->d_cu_map, 0, kCuKeys * sizeof(unsigned)));
    }
    if (on) HIP_TRY(hipMemset(h->d_phases, 0, kFirPhaseWords * sizeof(unsigned long long)));
    h->fir_phases = on != 0;
    return QPSK_OK;
}

int qpsk_demod_fir_phases(qpsk_demod *h, uint64_t *out, int32_t n) {
    if (!h || !out) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    if (n < kFirPhaseWords) return fail(QPSK_ERR_ARGUMENT, "n < 16");
    if (!h->d_phases) {
        std::memset(out, 0, kFirPhaseWords * sizeof(uint64_t));
        return kFirPhaseWords;
    }
    int rc;
    if ((rc = drain_async(h))) return rc;
    HIP_TRY(hipSetDevice(h->p.device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipMemcpy(out, h->d_phases, kFirPhaseWords * sizeof(uint64_t), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(h->d_phases, 0, kFirPhaseWords * sizeof(unsigned long long)));
    return kFirPhaseWords;
}

// per timed call: FLL, FIR and loop kernel durations and the call's kernel
// span (earliest start to latest end), ms; 0 for a kernel that did not run
static int read_launch_times(qpsk_demod *h, std::vector<float> *out) {
    out->assign(static_cast<size_t>(h->kt_used) * 4, 0.f);
    if (!h->kt_used) return QPSK_OK;
    int rc;
    if ((rc = drain_async(h))) return rc;
    HIP_TRY(hipSetDevice(h->p.device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (h->s_front) HIP_TRY(hipStreamSynchronize(h->s_front));
    if (h->s_back) HIP_TRY(hipStreamSynchronize(h->s_back));
    std::vector<unsigned long long> t(static_cast<size_t>(h->kt_used) * kKtPerCall);
    HIP_TRY(hipMemcpy(t.data(), h->d_kt, t.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    const double ms_per_tick = 1.0 / h->wall_khz;
    for (int c = 0; c < h->kt_used; ++c) {
        const unsigned long long *k = t.data() + static_cast<size_t>(kKtPerCall) * c;
        unsigned long long lo = ~0ull, hi = 0;
        for (int j = 0; j < 3; ++j) {
            const unsigned long long s0 = k[2 * j], e0 = k[2 * j + 1];
            if (s0 == ~0ull || e0 < s0) continue;   // did not run
            (*out)[4 * c + j] = static_cast<float>((e0 - s0) * ms_per_tick);
            lo = std::min(lo, s0);
            hi = std::max(hi, e0);
        }
        if (hi >= lo && lo != ~0ull) (*out)[4 * c + 3] = static_cast<float>((hi - lo) * ms_per_tick);
    }
    return QPSK_OK;
}

int qpsk_demod_stage_times(qpsk_demod *h, float *ms, int32_t n) {
    if (!h || !ms) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    std::vector<float> t;
    int rc;
    if ((rc = read_launch_times(h, &t))) return rc;
    const int k = std::min<int32_t>(n, 4);
    for (int i = 0; i < k; ++i) {
        double sum = 0;
        int cnt = 0;
        for (int c = 0; c < h->kt_used; ++c)
            if (t[4 * c + i] > 0.f) {
                sum += t[4 * c + i];
                ++cnt;
            }
        ms[i] = cnt ? static_cast<float>(sum / cnt) : 0.f;
    }
    return k;
}

int qpsk_demod_kernel_clocks(qpsk_demod *h, float *ghz, int32_t max_calls) {
    if (!h || !ghz) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    if (!h->kt_used) return 0;
    int rc;
    if ((rc = drain_async(h))) return rc;
    HIP_TRY(hipSetDevice(h->p.device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (h->s_front) HIP_TRY(hipStreamSynchronize(h->s_front));
    if (h->s_back) HIP_TRY(hipStreamSynchronize(h->s_back));
    std::vector<unsigned long long> t(static_cast<size_t>(h->kt_used) * kKtPerCall);
    HIP_TRY(hipMemcpy(t.data(), h->d_kt, t.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    const int k = std::min<int32_t>(max_calls, h->kt_used);
    for (int c = 0; c < k; ++c) {
        const unsigned long long *s = t.data() + static_cast<size_t>(kKtPerCall) * c;
        // FLL (slots 8, 9), FIR (6, 7), loop kernel (10, 11)
        const int slot[3] = {8, 6, 10};
        for (int j = 0; j < 3; ++j) {
            const unsigned long long cy = s[slot[j]], wt = s[slot[j] + 1];
            ghz[3 * c + j] = wt ? static_cast<float>(static_cast<double>(cy) / wt * h->wall_khz * 1e-6) : 0.f;
        }
    }
    return k;
}

int qpsk_demod_launch_times(qpsk_demod *h, float *ms, int32_t max_calls) {
    if (!h || !ms) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    std::vector<float> t;
    int rc;
    if ((rc = read_launch_times(h, &t))) return rc;
    const int k = std::min<int32_t>(max_calls, h->kt_used);
    std::memcpy(ms, t.data(), static_cast<size_t>(k) * 4 * sizeof(float));
    return k;
}

}  // extern "C"

namespace {

// One validated call of at most max_samples_per_call samples per stream.
int process_one(qpsk_demod *h, const Call &c) {
    int rc;
    const int32_t mem = c.mem;
    const float *iq = c.iq;
    const int64_t stride_floats = c.stride_floats;
    const int64_t *lengths = c.lengths;
    const int S = h->S;
    const int64_t n_call = c.n_call;
    hipStream_t st = h->stream;
    HIP_TRY(hipSetDevice(h->p.device));
    // pipelined calls issued before this one finish first (they share the state)
    if ((rc = flush_deferred(h))) return rc;
    if (hipEvent_t e = last_async(h)) HIP_TRY(hipStreamWaitEvent(st, e, 0));
    unsigned long long *kt = next_kt(h);
    if (mem == QPSK_MEM_HOST && !c.append) HIP_TRY(hipMemsetAsync(h->d_flags + 1, 0, sizeof(uint32_t), st));

    // ---- input -----------------------------------------------------------
    const float *x = iq;
    int64_t x_stride = stride_floats / 2;   // float2 units
    if (n_call > 0 && mem == QPSK_MEM_HOST) {
        if (!h->d_in && (rc = dev_alloc(&h->d_in, static_cast<size_t>(2 * S * h->n_max)))) return rc;
        HIP_TRY(hipMemcpy2DAsync(h->d_in, 2 * h->n_max * sizeof(float), iq, stride_floats * sizeof(float),
                                 2 * n_call * sizeof(float), S, hipMemcpyHostToDevice, st));
        x = h->d_in;
        x_stride = h->n_max;
    }
    const int64_t *d_len = nullptr;
    if (lengths) {
        HIP_TRY(hipMemcpyAsync(h->d_lengths[0], lengths, S * sizeof(int64_t), hipMemcpyHostToDevice, st));
        d_len = h->d_lengths[0];
    }

    if (h->p.iq_balance && n_call > 0) {
        run_iqb(h, x, x_stride, d_len, n_call, st);
        x = h->d_iqb;
        x_stride = h->n_max;
    }
    if (h->p.enable_fll && n_call > 0) {
        run_fll(h, x, x_stride, d_len, n_call, h->d_fll_out[0], st, kt);
        x = h->d_fll_out[0];
        x_stride = h->n_max;
    }
    if ((rc = run_fir(h, x, x_stride, d_len, n_call, h->d_mf[0], st, kt))) return rc;
    return run_loop(h, c, d_len, h->d_mf[0], st, kt);
}

int process_async_one(qpsk_demod *h, const Call &c) {
    int rc;
    const float *iq = c.iq;
    const int64_t stride_floats = c.stride_floats;
    const int64_t *lengths = c.lengths;
    HIP_TRY(hipSetDevice(h->p.device));
    if ((rc = pipe_setup(h))) return rc;
    const int S = h->S;
    const int64_t n_call = c.n_call;
    const int b = h->pipe_bufs == 2 ? h->pipe_cur : 0;
    h->pipe_cur ^= 1;
    hipStream_t F = h->s_front, B = h->s_back;

    // the front stage starts after the work already on the handle's stream
    // (the producer of iq, earlier synchronous calls) and after the back stage
    // that last used boundary buffer b
    HIP_TRY(hipEventRecord(h->e_in, h->stream));
    HIP_TRY(hipStreamWaitEvent(F, h->e_in, 0));
    const int prev = h->pipe_bufs == 2 ? b : h->last_back;
    if (prev >= 0 && h->back_rec[prev]) HIP_TRY(hipStreamWaitEvent(F, h->e_back[prev], 0));
    unsigned long long *kt = next_kt(h);
    const int64_t *d_len = nullptr;
    if (lengths) {
        // pinned staging row b is free once the front stage that last read it ran
        if (h->front_rec[b]) HIP_TRY(hipEventSynchronize(h->e_front[b]));
        std::memcpy(h->h_len[b], lengths, S * sizeof(int64_t));
        HIP_TRY(hipMemcpyAsync(h->d_lengths[b], h->h_len[b], S * sizeof(int64_t), hipMemcpyHostToDevice, F));
        d_len = h->d_lengths[b];
    }
    const float *x = iq;
    int64_t x_stride = stride_floats / 2;
    if (h->p.iq_balance && n_call > 0) {
        // read only by this call's own front stage (FLL or FIR on F)
        run_iqb(h, x, x_stride, d_len, n_call, F);
        x = h->d_iqb;
        x_stride = h->n_max;
    }
    float *mf;
    if (h->p.enable_fll) {
        // FLL on (C5): the FLL keeps every SIMD's VALU busy with one wave each
        // (DESIGN.md 3.3), so a kernel beside it gains what it takes from it,
        // and the launches swing (FIR 48-198, loop 23-218 ms at C5 in round 2).
        // The FIR and the loop kernel overlap well (the FLL-off pipeline).  So:
        //   F: FLL(k) alone -> [B: loop(k-1) after FLL(k)] -> F: FIR(k) once
        //   loop(k-1) holds its CUs (residency gate) -> FIR(k) || loop(k-1)
        // The loop kernel of call k is issued by call k+1 after its FLL, or by
        // a flush (pipeline_wait, a synchronous call, state access, destroy).
        // FLL(k) waited above for loop(k-2), the last reader of MF rows b, and
        // follows FIR(k-1) on F, so it runs alone.
        if (n_call > 0) run_fll(h, x, x_stride, d_len, n_call, h->d_fll_out[0], F, kt);
        HIP_TRY(hipEventRecord(h->e_fll, F));
        if (h->deferred) {
            Call dc = h->dcall;
            HIP_TRY(hipStreamWaitEvent(B, h->e_fll, 0));
            const int db = h->dbuf;
            h->deferred = false;
            if ((rc = run_loop(h, dc, h->dlen, h->d_mf[db], B, h->dkt, h->use_gate ? h->d_resident : nullptr)))
                return rc;
            HIP_TRY(hipEventRecord(h->e_back[db], B));
            h->back_rec[db] = true;
            h->last_back = db;
        }
        if ((rc = gate_wait(h, F))) return rc;
        mf = h->d_mf[b];
        if ((rc = run_fir(h, n_call > 0 ? h->d_fll_out[0] : x, n_call > 0 ? h->n_max : x_stride, d_len, n_call,
                          mf, F, kt)))
            return rc;
        HIP_TRY(hipEventRecord(h->e_front[b], F));
        h->front_rec[b] = true;
        h->dcall = c;
        h->dbuf = b;
        h->dlen = d_len;
        h->dkt = kt;
        h->deferred = true;
        // one MF buffer only: nothing can overlap, issue the back stage now
        return h->pipe_bufs == 2 ? QPSK_OK : flush_deferred(h);
    } else {
        // front = FIR into MF rows b; back = loop.  FIR(k+1) and loop(k) both
        // become ready when a stage of call k-1 or k ends, and whichever is
        // dispatched first takes the CUs: a loop kernel dispatched after the
        // FIR finds no CU with room for its 104-147 KB workgroups and runs
        // after it (measured on MI355X at C3 under rocprofv3: FIR 42 + loop
        // 80 ms a call, against FIR 52 || loop 43 the other way round,
        // profiles/archive/r02_c3_dispatch_race.txt; reproduced by
        // tools/anyorder_probe.hip), and either order then repeats call after
        // call.  So FIR(k+1) waits, on the device, until loop(k)'s workgroups
        // hold their CUs: each adds 1 to the residency counter as it starts,
        // and the front stream waits for the count (hipStreamWaitValue64 on
        // signal memory, gate_wait: bounded).  The order no longer depends on
        // dispatch timing: the FIR cannot be dispatched before min(grid, CUs)
        // loop workgroups run, and every one of those was dispatched before it.
        if ((rc = gate_wait(h, F))) return rc;
        mf = h->d_mf[b];
        if ((rc = run_fir(h, x, x_stride, d_len, n_call, mf, F, kt))) return rc;
        HIP_TRY(hipEventRecord(h->e_front[b], F));
        HIP_TRY(hipStreamWaitEvent(B, h->e_front[b], 0));
    }
    h->front_rec[b] = true;
    if ((rc = run_loop(h, c, d_len, mf, B, kt, h->use_gate ? h->d_resident : nullptr))) return rc;
    HIP_TRY(hipEventRecord(h->e_back[b], B));
    h->back_rec[b] = true;
    h->last_back = b;
    return QPSK_OK;
}

// The deferred back stage (FLL on) after its own FIR only: nothing follows it.
int flush_deferred(qpsk_demod *h) {
    if (!h->deferred) return QPSK_OK;
    HIP_TRY(hipSetDevice(h->p.device));
    const int db = h->dbuf;
    h->deferred = false;
    HIP_TRY(hipStreamWaitEvent(h->s_back, h->e_front[db], 0));
    int rc;
    if ((rc = run_loop(h, h->dcall, h->dlen, h->d_mf[db], h->s_back, h->dkt))) return rc;
    HIP_TRY(hipEventRecord(h->e_back[db], h->s_back));
    h->back_rec[db] = true;
    h->last_back = db;
    return QPSK_OK;
}

// QPSK_STATUS_* raised by the host-memory call that just finished -> status
int host_call_status(qpsk_demod *h) {
    const uint32_t f = *h->h_flags;
    if (f & QPSK_STATUS_CARRY_OVERFLOW)
        return fail(QPSK_ERR_STATE, "symbol-sync queue over 256 retained samples (output capacity hit: sps below ~1?)");
    if (f & QPSK_STATUS_OUTPUT_TRUNCATED) return fail(QPSK_ERR_CAPACITY, "output row truncated");
    if (f & QPSK_STATUS_NONFINITE_TIMING)
        return fail(QPSK_ERR_STATE, "non-finite sample reached the symbol timing loop");
    return QPSK_OK;
}

// A call longer than max_samples_per_call (QPSKDeModulator.cs:345-360 accepts
// any span): consecutive internal chunks of at most n_max samples per stream,
// each chunk's rows appended behind the previous one's, so the caller sees the
// output of one call (the chain carries its state across chunks exactly as
// across calls).  Host-memory outputs are staged in device rows of the whole
// call and copied back once.
int process_chunked(qpsk_demod *h, const Call &c, bool async) {
    const int S = h->S;
    const int64_t N = h->n_max;
    int rc;
    HIP_TRY(hipSetDevice(h->p.device));
    if (!h->d_acc && (rc = dev_alloc(&h->d_acc, 2 * static_cast<size_t>(S)))) return rc;
    if (c.syms && !h->d_syms && (rc = dev_alloc(&h->d_syms, static_cast<size_t>(2 * S * h->syms_cap))))
        return rc;
    const bool host = c.mem == QPSK_MEM_HOST;
    const int64_t bytes_row = (2 * c.max_sym + 7) / 8;
    uint8_t *dbits = c.bits;
    int64_t dbits_stride = c.bits_stride_bytes;
    float *dsyms = c.syms;
    int64_t dsyms_stride = c.syms_stride_floats;
    if (host) {
        if (async) return fail(QPSK_ERR_ARGUMENT, "pipelined calls take device memory");
        if (c.bits) {
            const size_t need = static_cast<size_t>(S) * bytes_row;
            if (need > h->xbits_bytes) {
                hipFree(h->d_xbits);
                h->d_xbits = nullptr;
                h->xbits_bytes = 0;
                if ((rc = dev_alloc(&h->d_xbits, need))) return rc;
                h->xbits_bytes = need;
            }
            dbits = h->d_xbits;
            dbits_stride = bytes_row;
        }
        if (c.syms) {
            const size_t need = static_cast<size_t>(S) * 2 * c.max_sym * sizeof(float);
            if (need > h->xsyms_bytes) {
                hipFree(h->d_xsyms);
                h->d_xsyms = nullptr;
                h->xsyms_bytes = 0;
                if ((rc = dev_alloc(&h->d_xsyms, need / sizeof(float)))) return rc;
                h->xsyms_bytes = need;
            }
            dsyms = h->d_xsyms;
            dsyms_stride = 2 * c.max_sym;
        }
        HIP_TRY(hipMemsetAsync(h->d_flags + 1, 0, sizeof(uint32_t), h->stream));
    }
    const int64_t K = (c.n_call + N - 1) / N;
    std::vector<int64_t> len_k(c.lengths ? S : 0);
    for (int64_t k = 0; k < K; ++k) {
        const int64_t off = k * N;
        Call sub = c;
        sub.iq = c.iq + 2 * off;
        if (c.lengths) {
            int64_t m = 0;
            for (int s = 0; s < S; ++s) {
                len_k[s] = std::min(N, std::max<int64_t>(0, c.lengths[s] - off));
                m = std::max(m, len_k[s]);
            }
            sub.lengths = len_k.data();
            sub.n_samples = 0;
            sub.n_call = m;
        } else {
            sub.n_samples = std::min(N, c.n_samples - off);
            sub.n_call = sub.n_samples;
        }
        sub.max_sym = qpsk_demod_max_symbols(h, sub.n_call);
        sub.append = true;
        sub.first = k == 0;
        sub.last = k == K - 1;
        sub.dst_bits = dbits;
        sub.dst_bits_stride = dbits_stride;
        sub.dst_syms = dsyms;
        sub.dst_syms_stride = dsyms_stride;
        sub.dst_n_bits = host ? nullptr : c.n_bits;
        sub.dst_n_syms = host ? nullptr : c.n_syms;
        if ((rc = async ? process_async_one(h, sub) : process_one(h, sub))) {
            // a chunk after the first failed: the chunks that ran left
            // StreamState.tofs (the queue offset inside this call) non-zero,
            // which only the last chunk resets; clear it so the next call's
            // timing runs from its own queue start (best effort after a HIP error)
            // The memset goes behind every kernel that may still write tofs:
            // the pipelined chunks' loop kernels run on the back stream, and
            // with the FLL the newest one is only issued by flush_deferred.
            if (k > 0) {
                (void)flush_deferred(h);
                if (hipEvent_t e = last_async(h)) (void)hipStreamWaitEvent(h->stream, e, 0);
                (void)hipMemset2DAsync(reinterpret_cast<char *>(h->d_state) + offsetof(StreamState, tofs),
                                       sizeof(StreamState), 0, sizeof(int64_t), S, h->stream);
            }
            return rc;
        }
    }
    if (!host) return QPSK_OK;
    hipStream_t st = h->stream;
    if (c.bits && bytes_row > 0)
        HIP_TRY(hipMemcpy2DAsync(c.bits, c.bits_stride_bytes, dbits, dbits_stride, bytes_row, S,
                                 hipMemcpyDeviceToHost, st));
    if (c.syms && c.max_sym > 0)
        HIP_TRY(hipMemcpy2DAsync(c.syms, c.syms_stride_floats * sizeof(float), dsyms,
                                 dsyms_stride * sizeof(float), 2 * c.max_sym * sizeof(float), S,
                                 hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(h->h_counts, h->d_acc, 2 * S * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(h->h_flags, h->d_flags + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (c.n_bits) std::memcpy(c.n_bits, h->h_counts, S * sizeof(int64_t));
    if (c.n_syms) std::memcpy(c.n_syms, h->h_counts + S, S * sizeof(int64_t));
    h->status_host |= *h->h_flags;
    return host_call_status(h);
}

}  // namespace (calls)

namespace qpsk {
// The host waits for every call queued on the handle, pipelined or stream-ordered
// (the multi-device group's join, qpsk_group.cpp).
int handle_sync(qpsk_demod *h) {
    int rc;
    if ((rc = drain_async(h))) return rc;
    HIP_TRY(hipSetDevice(h->p.device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return QPSK_OK;
}
}  // namespace qpsk

extern "C" {

int qpsk_demod_process(qpsk_demod *h, int32_t mode, const float *iq, int64_t stride_floats,
                       int64_t n_samples, const int64_t *lengths, int32_t mem, uint8_t *bits,
                       int64_t bits_stride_bytes, int64_t *n_bits, float *syms,
                       int64_t syms_stride_floats, int64_t *n_syms) {
    Call c{mode, iq, stride_floats, n_samples, lengths, mem, bits, bits_stride_bytes, n_bits,
           syms, syms_stride_floats, n_syms};
    int rc;
    if ((rc = validate(h, c))) return rc;
    if (c.n_call > h->n_max) return process_chunked(h, c, false);
    if ((rc = process_one(h, c))) return rc;
    return c.mem == QPSK_MEM_HOST ? host_call_status(h) : QPSK_OK;
}

int qpsk_demod_process_async(qpsk_demod *h, int32_t mode, const float *iq, int64_t stride_floats,
                             int64_t n_samples, const int64_t *lengths, uint8_t *bits,
                             int64_t bits_stride_bytes, int64_t *n_bits, float *syms,
                             int64_t syms_stride_floats, int64_t *n_syms) {
    Call c{mode, iq, stride_floats, n_samples, lengths, QPSK_MEM_DEVICE, bits, bits_stride_bytes,
           n_bits, syms, syms_stride_floats, n_syms};
    int rc;
    if ((rc = validate(h, c))) return rc;
    if (c.n_call > h->n_max) return process_chunked(h, c, true);
    return process_async_one(h, c);
}

int qpsk_demod_last_mf(qpsk_demod *h, float *out, int64_t stride_floats, int64_t n_samples, int32_t mem) {
    if (!h || !out) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    if (n_samples < 0 || n_samples > h->n_max || stride_floats < 2 * n_samples)
        return fail(QPSK_ERR_ARGUMENT, "n_samples / stride_floats out of range");
    if (mem != QPSK_MEM_HOST && mem != QPSK_MEM_DEVICE) return fail(QPSK_ERR_ARGUMENT, "unknown mem");
    HIP_TRY(hipSetDevice(h->p.device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (n_samples == 0) return QPSK_OK;
    HIP_TRY(hipMemcpy2D(out, stride_floats * sizeof(float), h->d_mf[0] + 2 * kMfPrefix,
                        2 * h->mf_stride * sizeof(float), 2 * n_samples * sizeof(float), h->S,
                        mem == QPSK_MEM_HOST ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice));
    return QPSK_OK;
}

int qpsk_demod_status(qpsk_demod *h, uint32_t *flags) {
    if (!h || !flags) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    int rc;
    if ((rc = drain_async(h))) return rc;
    HIP_TRY(hipSetDevice(h->p.device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipMemcpy(h->h_flags, h->d_flags, sizeof(uint32_t), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(h->d_flags, 0, sizeof(uint32_t)));
    *flags = *h->h_flags | h->status_host;
    h->status_host = 0;
    return QPSK_OK;
}

int qpsk_demod_pipeline_wait(qpsk_demod *h, void *hip_stream) {
    if (!h) return fail(QPSK_ERR_ARGUMENT_NULL, "null handle");
    int rc;
    if ((rc = flush_deferred(h))) return rc;
    hipEvent_t e = last_async(h);
    if (!e) return QPSK_OK;
    if (hip_stream) HIP_TRY(hipStreamWaitEvent(static_cast<hipStream_t>(hip_stream), e, 0));
    else HIP_TRY(hipEventSynchronize(e));
    return QPSK_OK;
}

int qpsk_demod_gate_timeouts(qpsk_demod *h, uint64_t *count) {
    if (!h || !count) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    *count = 0;
    if (!h->d_gate) return QPSK_OK;
    int rc;
    if ((rc = drain_async(h))) return rc;
    HIP_TRY(hipSetDevice(h->p.device));
    unsigned v = 0;
    HIP_TRY(hipMemcpy(&v, h->d_gate, sizeof(unsigned), hipMemcpyDeviceToHost));
    *count = v;
    return QPSK_OK;
}

int qpsk_demod_pipeline_depth(const qpsk_demod *h) {
    if (!h) return fail(QPSK_ERR_ARGUMENT_NULL, "null handle");
    return h->pipe_ready ? h->pipe_bufs : 0;
}

int qpsk_demod_rrc_taps(const qpsk_demod *h, float *taps, int32_t cap) {
    if (!h || !taps) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    if (cap < h->T) return fail(QPSK_ERR_ARGUMENT, "cap too small");
    std::memcpy(taps, h->d.rrc_f32.data(), h->T * sizeof(float));
    return h->T;
}

int qpsk_demod_gains(const qpsk_demod *h, double *mm_sps, double *kp, double *ki,
                     double *costas_alpha, double *costas_beta) {
    if (!h) return fail(QPSK_ERR_ARGUMENT_NULL, "null handle");
    if (mm_sps) *mm_sps = h->d.mm_sps;
    if (kp) *kp = h->d.kp;
    if (ki) *ki = h->d.ki;
    if (costas_alpha) *costas_alpha = h->d.costas_alpha;
    if (costas_beta) *costas_beta = h->d.costas_beta;
    return QPSK_OK;
}

int qpsk_demod_fll_taps(const qpsk_demod *h, float *lower_iq, float *upper_iq, int32_t cap_floats) {
    if (!h || !lower_iq || !upper_iq) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    const int n = 2 * kFllTaps;
    if (cap_floats < n) return fail(QPSK_ERR_ARGUMENT, "cap too small");
    std::memcpy(lower_iq, h->d.fll_lower_iq.data(), n * sizeof(float));
    std::memcpy(upper_iq, h->d.fll_upper_iq.data(), n * sizeof(float));
    return n;
}

int qpsk_demod_design(const qpsk_demod_params *p, float *rrc_taps, int32_t cap, double *gains,
                      float *fll_lower_iq, float *fll_upper_iq) {
    if (!p) return fail(QPSK_ERR_ARGUMENT_NULL, "null params");
    LoopDesign d;
    std::string err;
    int rc = design_loops(p->sample_rate, p->symbol_rate, p->rrc_alpha, p->rrc_span,
                          p->symbol_sync_bandwidth, p->costas_loop_bandwidth, p->cfo_loop_bandwidth,
                          &d, &err);
    if (rc != QPSK_OK) return fail(rc, err);
    const int T = static_cast<int>(d.rrc_f32.size());
    if (rrc_taps) {
        if (cap < T) return fail(QPSK_ERR_ARGUMENT, "cap too small");
        std::memcpy(rrc_taps, d.rrc_f32.data(), T * sizeof(float));
    }
    if (gains) {
        gains[0] = d.mm_sps; gains[1] = d.kp; gains[2] = d.ki;
        gains[3] = d.costas_alpha; gains[4] = d.costas_beta;
    }
    if (fll_lower_iq) std::memcpy(fll_lower_iq, d.fll_lower_iq.data(), 2 * kFllTaps * sizeof(float));
    if (fll_upper_iq) std::memcpy(fll_upper_iq, d.fll_upper_iq.data(), 2 * kFllTaps * sizeof(float));
    return T;
}

// State blob (format 2): a header naming the layout, then the per-stream
// records, the M&M carries, the FIR histories and the FLL delay lines.  Format
// 1 (round 3 and before) had no header and a 64-sample carry; set_state
// rejects any blob whose header or length does not match this handle.
namespace {
constexpr uint32_t kStateMagic = 0x4b535051u;   // "QPSK"
constexpr uint32_t kStateFormat = 2;
struct StateHeader {
    uint32_t magic, format;
    int32_t streams, taps, carry_max, fll_taps, record_bytes, reserved;
};
static_assert(sizeof(StateHeader) == 32, "state blob header");
StateHeader state_header(const qpsk_demod *h) {
    return StateHeader{kStateMagic, kStateFormat, h->S, h->T, kCarryMax, kFllTaps,
                       static_cast<int32_t>(sizeof(StreamState)), 0};
}
}  // namespace

int64_t qpsk_demod_state_bytes(const qpsk_demod *h) {
    if (!h) return 0;
    const int64_t S = h->S, H = h->T - 1;
    return static_cast<int64_t>(sizeof(StateHeader)) +
           S * (static_cast<int64_t>(sizeof(StreamState)) + 8 * kCarryMax + 8 * H + 8 * 2 * kFllTaps);
}

int qpsk_demod_get_state(qpsk_demod *h, void *host_buf, int64_t buf_bytes) {
    if (!h || !host_buf) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    if (buf_bytes < qpsk_demod_state_bytes(h)) return fail(QPSK_ERR_ARGUMENT, "state buffer too small");
    const int64_t S = h->S, H = h->T - 1;
    char *p = static_cast<char *>(host_buf);
    int rc;
    if ((rc = drain_async(h))) return rc;
    HIP_TRY(hipSetDevice(h->p.device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    const StateHeader hd = state_header(h);
    std::memcpy(p, &hd, sizeof(hd));
    p += sizeof(hd);
    HIP_TRY(hipMemcpy(p, h->d_state, S * sizeof(StreamState), hipMemcpyDeviceToHost));
    p += S * sizeof(StreamState);
    HIP_TRY(hipMemcpy(p, h->d_carry, S * 8 * kCarryMax, hipMemcpyDeviceToHost));
    p += S * 8 * kCarryMax;
    if (H > 0) HIP_TRY(hipMemcpy(p, h->d_hist[h->hist_cur], S * 8 * H, hipMemcpyDeviceToHost));
    p += S * 8 * H;
    HIP_TRY(hipMemcpy(p, h->d_fll_delay, S * 8 * 2 * kFllTaps, hipMemcpyDeviceToHost));
    return QPSK_OK;
}

int qpsk_demod_set_state(qpsk_demod *h, const void *host_buf, int64_t buf_bytes) {
    if (!h || !host_buf) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    if (buf_bytes != qpsk_demod_state_bytes(h))
        return fail(QPSK_ERR_ARGUMENT, "state blob length does not match this handle (" +
                                           std::to_string(buf_bytes) + " vs " +
                                           std::to_string(qpsk_demod_state_bytes(h)) + " bytes)");
    const StateHeader want = state_header(h);
    StateHeader got;
    std::memcpy(&got, host_buf, sizeof(got));
    if (got.magic != want.magic || got.format != want.format)
        return fail(QPSK_ERR_ARGUMENT, "not a state blob of this library version (format " +
                                           std::to_string(got.format) + ", expected " +
                                           std::to_string(want.format) + ")");
    if (got.streams != want.streams || got.taps != want.taps || got.carry_max != want.carry_max ||
        got.fll_taps != want.fll_taps || got.record_bytes != want.record_bytes)
        return fail(QPSK_ERR_ARGUMENT, "state blob layout (streams, taps, carry, record size) does not "
                                       "match this handle");
    const int64_t S = h->S, H = h->T - 1;
    const char *p = static_cast<const char *>(host_buf) + sizeof(StateHeader);
    int rc;
    if ((rc = drain_async(h))) return rc;
    HIP_TRY(hipSetDevice(h->p.device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipMemcpy(h->d_state, p, S * sizeof(StreamState), hipMemcpyHostToDevice));
    p += S * sizeof(StreamState);
    HIP_TRY(hipMemcpy(h->d_carry, p, S * 8 * kCarryMax, hipMemcpyHostToDevice));
    p += S * 8 * kCarryMax;
    if (H > 0) HIP_TRY(hipMemcpy(h->d_hist[h->hist_cur], p, S * 8 * H, hipMemcpyHostToDevice));
    p += S * 8 * H;
    HIP_TRY(hipMemcpy(h->d_fll_delay, p, S * 8 * 2 * kFllTaps, hipMemcpyHostToDevice));
    return QPSK_OK;
}

int32_t qpsk_demod_pick_loop_variant(int32_t requested, int32_t n_streams, double sps, int32_t cus) {
    if (requested != 0 || !(sps >= 8.0) || cus <= 0 || n_streams <= 0) return requested;
    const int64_t S = n_streams;
    if ((S + 5) / 6 <= cus) return 7;
    if ((S + 11) / 12 <= cus) return 6;
    return 0;
}

// Residency gate default (process_async_one).  The wait is bounded
// (gate_wait_kernel), but where dispatch is serialised the loop kernel it
// waits for starts only after the waiting FIR, so every wait would run to its
// cap: the gate is off there.
int qpsk_pipeline_gate_enabled(void) {
    auto env = [](const char *name) -> const char * {
        const char *v = std::getenv(name);
        return v && *v ? v : nullptr;
    };
    auto is = [&](const char *name, const char *val) {
        const char *v = env(name);
        return v && std::strcmp(v, val) == 0;
    };
    auto nonzero = [&](const char *name) {
        const char *v = env(name);
        return v && std::strcmp(v, "0") != 0;
    };
    if (is("QPSK_PIPELINE_GATE", "0")) return 0;             // explicit opt-out
    if (is("QPSK_PIPELINE_GATE", "1")) return 1;             // explicit opt-in wins over the rest
    if (nonzero("AMD_SERIALIZE_KERNEL")) return 0;           // HIP runtime: serialised kernel launches
    if (nonzero("AMD_SERIALIZE_COPY")) return 0;             // ... and copies
    if (nonzero("HIP_LAUNCH_BLOCKING")) return 0;            // every launch waits for the previous
    if (nonzero("CUDA_LAUNCH_BLOCKING")) return 0;           // the alias HIP also honours
    if (is("ROCPROF_COUNTER_COLLECTION", "1")) return 0;     // rocprofv3 --pmc: per-dispatch serialisation
    if (nonzero("ROCPROFILER_KERNEL_SERIALIZATION")) return 0;
    if (nonzero("HSA_ENABLE_DEBUG")) return 0;               // debugger-attached runs
    return 1;
}

}  // extern "C"
