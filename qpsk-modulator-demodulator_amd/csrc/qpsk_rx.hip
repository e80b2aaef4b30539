// qpsk_rx.hip -- host-fed streaming front-end.
//
// The reference's deployment loop (ModDemodOverSDR.cs:116-183) reads CF32
// buffers from the SDR and calls DeModulate on each in turn, one host thread,
// state carried from call to call.  Here a ring of `depth` pinned host slots
// feeds one batched handle:
//
//   submit k:  [host copy into pinned slot k%D unless the caller filled it]
//              upload stream U : wait(slot free) -> H2D slot -> (handle's stream)
//              qpsk_demod_process_async: front (FIR / FLL) then back (loop)
//              front stream    : record in_free[slot]   (input consumed)
//              download stream : wait(back stage) -> D2H bits, counts -> out_done[slot]
//   collect:   wait out_done of the oldest chunk, copy its rows to the caller
//
// U is the handle's own stream, so process_async's front stage is ordered
// after the upload; the next upload (slot k+1) only waits for the stage that
// last read ITS slot, so it runs on the copy engine while chunk k computes.
// Everything the chain computes is done by the same kernels in the same call
// order as synchronous qpsk_demod_process calls, hence identical bits.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "qpsk_demod.h"

namespace qpsk {
int set_last_error(int code, const std::string &msg);
hipStream_t pipe_front_stream(const qpsk_demod *h);
int handle_streams(const qpsk_demod *h);
int64_t handle_max_samples(const qpsk_demod *h);
int handle_device(const qpsk_demod *h);
}  // namespace qpsk

namespace {
int fail(int code, const std::string &msg) { return qpsk::set_last_error(code, msg); }

#define RX_TRY(expr)                                                                   \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return fail(QPSK_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct Slot {
    float *h_in = nullptr;      // pinned [S][in_stride]
    float *d_in = nullptr;      // device, same layout
    uint8_t *d_bits = nullptr;  // device [S][bits_stride]
    int64_t *d_nb = nullptr;    // device [S]
    uint8_t *h_bits = nullptr;  // pinned
    int64_t *h_nb = nullptr;    // pinned
    hipEvent_t in_free = nullptr, out_done = nullptr;
    bool in_rec = false, out_rec = false;
    int64_t row_bytes = 0;      // bit bytes per row this chunk can hold
};
}  // namespace

struct qpsk_rx {
    qpsk_demod *h = nullptr;
    int depth = 0;
    int S = 0;
    int64_t n_max = 0;
    int64_t in_stride = 0;      // floats
    int64_t bits_stride = 0;    // bytes
    int device = 0;
    hipStream_t up = nullptr, down = nullptr;
    std::vector<Slot> slots;
    int64_t submitted = 0, collected = 0;
};

namespace {
void release(qpsk_rx *r) {
    for (auto &s : r->slots) {
        if (s.h_in) hipHostFree(s.h_in);
        if (s.h_bits) hipHostFree(s.h_bits);
        if (s.h_nb) hipHostFree(s.h_nb);
        if (s.d_in) hipFree(s.d_in);
        if (s.d_bits) hipFree(s.d_bits);
        if (s.d_nb) hipFree(s.d_nb);
        if (s.in_free) hipEventDestroy(s.in_free);
        if (s.out_done) hipEventDestroy(s.out_done);
    }
    if (r->up) hipStreamDestroy(r->up);
    if (r->down) hipStreamDestroy(r->down);
    delete r;
}

int setup(qpsk_rx *r) {
    RX_TRY(hipSetDevice(r->device));
    RX_TRY(hipStreamCreateWithFlags(&r->up, hipStreamNonBlocking));
    RX_TRY(hipStreamCreateWithFlags(&r->down, hipStreamNonBlocking));
    const size_t S = static_cast<size_t>(r->S);
    const size_t in_bytes = S * static_cast<size_t>(r->in_stride) * sizeof(float);
    const size_t bit_bytes = S * static_cast<size_t>(r->bits_stride);
    r->slots.resize(r->depth);
    for (auto &s : r->slots) {
        RX_TRY(hipHostMalloc(reinterpret_cast<void **>(&s.h_in), in_bytes));
        RX_TRY(hipHostMalloc(reinterpret_cast<void **>(&s.h_bits), bit_bytes));
        RX_TRY(hipHostMalloc(reinterpret_cast<void **>(&s.h_nb), S * sizeof(int64_t)));
        RX_TRY(hipMalloc(reinterpret_cast<void **>(&s.d_in), in_bytes));
        RX_TRY(hipMalloc(reinterpret_cast<void **>(&s.d_bits), bit_bytes));
        RX_TRY(hipMalloc(reinterpret_cast<void **>(&s.d_nb), S * sizeof(int64_t)));
        RX_TRY(hipEventCreateWithFlags(&s.in_free, hipEventDisableTiming));
        RX_TRY(hipEventCreateWithFlags(&s.out_done, hipEventDisableTiming));
    }
    return QPSK_OK;
}
}  // namespace

extern "C" {

int qpsk_rx_create(qpsk_demod *h, int32_t depth, qpsk_rx **out) {
    if (!h || !out) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    *out = nullptr;
    if (depth < 2 || depth > 8) return fail(QPSK_ERR_ARGUMENT, "depth must be 2..8");
    qpsk_rx *r = new qpsk_rx;
    r->h = h;
    r->depth = depth;
    r->S = qpsk::handle_streams(h);
    r->n_max = qpsk::handle_max_samples(h);
    r->device = qpsk::handle_device(h);
    r->in_stride = 2 * r->n_max;
    r->bits_stride = ((2 * qpsk_demod_max_symbols(h, r->n_max) + 7) / 8 + 15) / 16 * 16;
    int rc = setup(r);
    if (rc == QPSK_OK) rc = qpsk_demod_set_stream(h, r->up);
    if (rc != QPSK_OK) {
        release(r);
        return rc;
    }
    *out = r;
    return QPSK_OK;
}

int qpsk_rx_destroy(qpsk_rx *r) {
    if (!r) return fail(QPSK_ERR_ARGUMENT_NULL, "null ring");
    hipSetDevice(r->device);
    qpsk_demod_pipeline_wait(r->h, nullptr);
    hipStreamSynchronize(r->up);
    hipStreamSynchronize(r->down);
    const int rc = qpsk_demod_set_stream(r->h, nullptr);
    release(r);
    return rc;
}

int qpsk_rx_next_slot(qpsk_rx *r, float **iq, int64_t *stride_floats) {
    if (!r || !iq) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    if (r->submitted - r->collected >= r->depth)
        return fail(QPSK_ERR_STATE, "every ring slot holds an uncollected chunk");
    Slot &sl = r->slots[r->submitted % r->depth];
    // the caller writes the slot next: its previous chunk must have been read
    if (sl.in_rec) RX_TRY(hipEventSynchronize(sl.in_free));
    *iq = sl.h_in;
    if (stride_floats) *stride_floats = r->in_stride;
    return QPSK_OK;
}

int qpsk_rx_submit(qpsk_rx *r, const float *iq, int64_t stride_floats, int64_t n_samples,
                   const int64_t *lengths, int64_t *ticket) {
    if (!r) return fail(QPSK_ERR_ARGUMENT_NULL, "null ring");
    if (r->submitted - r->collected >= r->depth)
        return fail(QPSK_ERR_STATE, "every ring slot holds an uncollected chunk");
    const int S = r->S;
    int64_t n_call = n_samples;
    if (lengths) {
        n_call = 0;
        for (int s = 0; s < S; ++s) {
            if (lengths[s] < 0) return fail(QPSK_ERR_ARGUMENT, "negative length");
            n_call = std::max(n_call, lengths[s]);
        }
    } else if (n_samples < 0) {
        return fail(QPSK_ERR_ARGUMENT, "negative n_samples");
    }
    if (n_call > r->n_max) return fail(QPSK_ERR_ARGUMENT, "chunk longer than the ring slots (max_samples_per_call)");
    if (n_call > 0 && !iq) return fail(QPSK_ERR_ARGUMENT_NULL, "SamplesIQ is null");
    if (n_call > 0 && stride_floats < 2 * n_call) return fail(QPSK_ERR_ARGUMENT, "stride too small");
    RX_TRY(hipSetDevice(r->device));
    Slot &sl = r->slots[r->submitted % r->depth];
    // the slot's previous chunk: its input was consumed (front stage) and its
    // bits were downloaded before this chunk overwrites either (the back stage
    // of this chunk follows the upload through the handle's stream)
    if (sl.in_rec) RX_TRY(hipEventSynchronize(sl.in_free));
    if (n_call > 0 && iq != sl.h_in) {
        for (int s = 0; s < S; ++s) {
            const int64_t len = lengths ? lengths[s] : n_call;
            std::memcpy(sl.h_in + static_cast<int64_t>(s) * r->in_stride, iq + static_cast<int64_t>(s) * stride_floats,
                        static_cast<size_t>(2 * len) * sizeof(float));
        }
    } else if (n_call > 0 && stride_floats != r->in_stride) {
        return fail(QPSK_ERR_ARGUMENT, "a ring slot has stride_floats = 2 * max_samples_per_call");
    }
    if (sl.out_rec) RX_TRY(hipStreamWaitEvent(r->up, sl.out_done, 0));
    if (n_call > 0)
        RX_TRY(hipMemcpy2DAsync(sl.d_in, r->in_stride * sizeof(float), sl.h_in, r->in_stride * sizeof(float),
                                2 * n_call * sizeof(float), S, hipMemcpyHostToDevice, r->up));
    int rc = qpsk_demod_process_async(r->h, QPSK_MODE_DEMODULATE, sl.d_in, r->in_stride, n_samples, lengths,
                                      sl.d_bits, r->bits_stride, sl.d_nb, nullptr, 0, nullptr);
    if (rc != QPSK_OK) return rc;
    RX_TRY(hipEventRecord(sl.in_free, qpsk::pipe_front_stream(r->h)));
    sl.in_rec = true;
    if ((rc = qpsk_demod_pipeline_wait(r->h, r->down)) != QPSK_OK) return rc;
    sl.row_bytes = (2 * qpsk_demod_max_symbols(r->h, n_call) + 7) / 8;
    RX_TRY(hipMemcpyAsync(sl.h_nb, sl.d_nb, S * sizeof(int64_t), hipMemcpyDeviceToHost, r->down));
    if (sl.row_bytes > 0)
        RX_TRY(hipMemcpy2DAsync(sl.h_bits, r->bits_stride, sl.d_bits, r->bits_stride, sl.row_bytes, S,
                                hipMemcpyDeviceToHost, r->down));
    RX_TRY(hipEventRecord(sl.out_done, r->down));
    sl.out_rec = true;
    if (ticket) *ticket = r->submitted;
    ++r->submitted;
    return QPSK_OK;
}

int qpsk_rx_collect(qpsk_rx *r, uint8_t *bits, int64_t bits_stride_bytes, int64_t *n_bits,
                    int64_t *ticket) {
    if (!r || !bits || !n_bits) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    if (r->collected == r->submitted) return fail(QPSK_ERR_STATE, "no chunk outstanding");
    Slot &sl = r->slots[r->collected % r->depth];
    if (bits_stride_bytes < sl.row_bytes)
        return fail(QPSK_ERR_ARGUMENT, "bits_stride_bytes smaller than 2*max_symbols/8");
    RX_TRY(hipSetDevice(r->device));
    RX_TRY(hipEventSynchronize(sl.out_done));
    for (int s = 0; s < r->S; ++s) {
        const int64_t nb = sl.h_nb[s];
        n_bits[s] = nb;
        std::memcpy(bits + static_cast<int64_t>(s) * bits_stride_bytes, sl.h_bits + static_cast<int64_t>(s) * r->bits_stride,
                    static_cast<size_t>((nb + 7) / 8));
    }
    if (ticket) *ticket = r->collected;
    ++r->collected;
    return QPSK_OK;
}

}  // extern "C"
