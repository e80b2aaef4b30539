// qpsk_group.cpp -- one batch of streams over several GPUs behind the C ABI
// (include/qpsk_demod.h "Multi-GPU group").
//
// Every reference QPSKDeModulator instance owns all of its loop state
// (QPSKDeModulator.cs:20-73, MuellerMuller.cs:24-36, CostasLoopQpsk.cs:25-27),
// so S independent streams split into contiguous shards with no exchange at
// all: shard k = streams [S*k/n, S*(k+1)/n) on devices[k], one ordinary handle
// each.  A group call fans the caller's rows out by row offset -- shard k reads
// iq + first_k * stride and writes bits + first_k * bits_stride, n_bits +
// first_k, ... -- and joins.  Each shard runs in its own persistent worker
// thread (a host-memory process() is synchronous and its H2D / D2H copies hold
// the thread), so the devices' calls, copies included, overlap.  Results are
// those of one handle over the whole batch, stream for stream: nothing a
// stream computes depends on which rows share its handle.
//
// No data-path collective: the shards never exchange samples.  RCCL
// scatter/gather of device-resident batches lives with torch.distributed in
// bench.py (one process per GPU); this is the one-process shape a C# host
// reaches through P/Invoke.
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "qpsk_demod.h"

namespace qpsk {
int set_last_error(int code, const std::string &msg);
int handle_sync(qpsk_demod *h);
int handle_device(const qpsk_demod *h);
}  // namespace qpsk

namespace {
int fail(int code, const std::string &msg) { return qpsk::set_last_error(code, msg); }

struct Shard {
    int32_t first = 0, count = 0, device = 0;
    qpsk_demod *h = nullptr;
};
}  // namespace

struct qpsk_demod_group {
    int32_t S = 0;
    std::vector<Shard> shards;
    // worker pool: worker k runs job(k) for every generation, then counts down
    std::vector<std::thread> threads;
    std::mutex m;
    std::condition_variable cv_go, cv_done;
    uint64_t gen = 0;
    int pending = 0;
    bool quit = false;
    std::function<int(int)> job;
    std::vector<int> rc;
    std::vector<std::string> err;
};

namespace {

void worker(qpsk_demod_group *g, int k) {
    uint64_t seen = 0;
    for (;;) {
        std::function<int(int)> job;
        {
            std::unique_lock<std::mutex> lk(g->m);
            g->cv_go.wait(lk, [&] { return g->quit || g->gen != seen; });
            if (g->quit) return;
            seen = g->gen;
            job = g->job;
        }
        const int rc = job(k);
        // the error text is thread-local: carry it back to the caller's thread
        std::string msg = rc < 0 ? std::string(qpsk_last_error()) : std::string();
        std::lock_guard<std::mutex> lk(g->m);
        g->rc[k] = rc;
        g->err[k] = std::move(msg);
        if (--g->pending == 0) g->cv_done.notify_all();
    }
}

// Run job(k) on every shard's worker and wait for all of them.  Returns the
// first failing shard's status (its message, prefixed with the shard, becomes
// this thread's qpsk_last_error); the other shards' calls still ran.
int fan_out(qpsk_demod_group *g, std::function<int(int)> job) {
    const int n = static_cast<int>(g->shards.size());
    {
        std::lock_guard<std::mutex> lk(g->m);
        g->job = std::move(job);
        g->pending = n;
        for (int k = 0; k < n; ++k) {
            g->rc[k] = QPSK_OK;
            g->err[k].clear();
        }
        ++g->gen;
    }
    g->cv_go.notify_all();
    std::unique_lock<std::mutex> lk(g->m);
    g->cv_done.wait(lk, [&] { return g->pending == 0; });
    for (int k = 0; k < n; ++k)
        if (g->rc[k] < 0)
            return fail(g->rc[k], "shard " + std::to_string(k) + " (device " +
                                      std::to_string(g->shards[k].device) + "): " + g->err[k]);
    return QPSK_OK;
}

void stop_workers(qpsk_demod_group *g) {
    {
        std::lock_guard<std::mutex> lk(g->m);
        g->quit = true;
    }
    g->cv_go.notify_all();
    for (auto &t : g->threads)
        if (t.joinable()) t.join();
    g->threads.clear();
}

}  // namespace

extern "C" {

int qpsk_shard_streams(int32_t n_streams, int32_t n_parts, int32_t k, int32_t *first, int32_t *count) {
    if (!first || !count) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    if (n_streams < 0 || n_parts <= 0 || k < 0 || k >= n_parts)
        return fail(QPSK_ERR_ARGUMENT, "need n_streams >= 0 and 0 <= k < n_parts");
    // the same split as bench.py shard_streams: lo = S*k/n, hi = S*(k+1)/n
    const int64_t S = n_streams;
    const int64_t lo = S * k / n_parts, hi = S * (k + 1) / n_parts;
    *first = static_cast<int32_t>(lo);
    *count = static_cast<int32_t>(hi - lo);
    return QPSK_OK;
}

int qpsk_demod_group_create(const qpsk_demod_params *p, const int32_t *devices, int32_t n_dev,
                            int32_t n_streams, qpsk_demod_group **out) {
    if (!p || !devices || !out) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    *out = nullptr;
    if (n_dev <= 0 || n_dev > 64) return fail(QPSK_ERR_ARGUMENT, "n_dev must be 1..64");
    if (n_streams < n_dev) return fail(QPSK_ERR_ARGUMENT, "n_streams must be >= n_dev (no empty shard)");
    for (int k = 0; k < n_dev; ++k)
        if (devices[k] < 0) return fail(QPSK_ERR_ARGUMENT, "negative device ordinal");
    auto *g = new qpsk_demod_group();
    g->S = n_streams;
    g->shards.resize(n_dev);
    g->rc.assign(n_dev, QPSK_OK);
    g->err.assign(n_dev, std::string());
    for (int k = 0; k < n_dev; ++k) {
        Shard &sh = g->shards[k];
        qpsk_shard_streams(n_streams, n_dev, k, &sh.first, &sh.count);
        sh.device = devices[k];
    }
    for (int k = 0; k < n_dev; ++k) g->threads.emplace_back(worker, g, k);
    // each shard's handle is made on its own worker thread: the devices
    // allocate and clear their (up to ~100 GB) buffers at the same time, and
    // the caller's current device is left alone
    const qpsk_demod_params base = *p;
    int rc = fan_out(g, [g, base](int k) {
        qpsk_demod_params q = base;
        q.device = g->shards[k].device;
        return qpsk_demod_create(&q, g->shards[k].count, &g->shards[k].h);
    });
    if (rc != QPSK_OK) {
        const std::string msg = qpsk_last_error();
        qpsk_demod_group_destroy(g);
        return fail(rc, msg);
    }
    *out = g;
    return QPSK_OK;
}

int qpsk_demod_group_destroy(qpsk_demod_group *g) {
    if (!g) return QPSK_OK;
    if (!g->threads.empty()) {
        // handles go on their workers too (each waits for its device's work)
        fan_out(g, [g](int k) {
            const int rc = qpsk_demod_destroy(g->shards[k].h);
            g->shards[k].h = nullptr;
            return rc;
        });
        stop_workers(g);
    }
    delete g;
    return QPSK_OK;
}

int qpsk_demod_group_size(const qpsk_demod_group *g) {
    if (!g) return fail(QPSK_ERR_ARGUMENT_NULL, "null group");
    return static_cast<int>(g->shards.size());
}

int qpsk_demod_group_shard(const qpsk_demod_group *g, int32_t k, int32_t *first_stream, int32_t *n_streams,
                           int32_t *device, qpsk_demod **handle) {
    if (!g) return fail(QPSK_ERR_ARGUMENT_NULL, "null group");
    if (k < 0 || k >= static_cast<int32_t>(g->shards.size())) return fail(QPSK_ERR_ARGUMENT, "no such shard");
    const Shard &sh = g->shards[k];
    if (first_stream) *first_stream = sh.first;
    if (n_streams) *n_streams = sh.count;
    if (device) *device = sh.device;
    if (handle) *handle = sh.h;
    return QPSK_OK;
}

int qpsk_demod_group_process(qpsk_demod_group *g, int32_t mode, const float *iq, int64_t stride_floats,
                             int64_t n_samples, const int64_t *lengths, int32_t mem, uint8_t *bits,
                             int64_t bits_stride_bytes, int64_t *n_bits, float *syms, int64_t syms_stride_floats,
                             int64_t *n_syms) {
    if (!g) return fail(QPSK_ERR_ARGUMENT_NULL, "null group");
    if (mode != QPSK_MODE_DEMODULATE && mode != QPSK_MODE_CONSTELLATION) return fail(QPSK_ERR_ARGUMENT, "unknown mode");
    if (mem != QPSK_MEM_HOST && mem != QPSK_MEM_DEVICE) return fail(QPSK_ERR_ARGUMENT, "unknown mem");
    // the checks every shard would make, made once on the whole batch first, so
    // a bad argument fails the call before any shard's state moves
    int64_t n_call = 0;
    if (lengths) {   // host memory in every call, as for qpsk_demod_process
        for (int s = 0; s < g->S; ++s) {
            if (lengths[s] < 0) return fail(QPSK_ERR_ARGUMENT, "negative length");
            n_call = lengths[s] > n_call ? lengths[s] : n_call;
        }
    } else {
        if (n_samples < 0) return fail(QPSK_ERR_ARGUMENT, "negative n_samples");
        n_call = n_samples;
    }
    if (n_call > 0 && !iq) return fail(QPSK_ERR_ARGUMENT_NULL, "SamplesIQ is null");
    if (n_call > 0 && stride_floats < 2 * n_call) return fail(QPSK_ERR_ARGUMENT, "stride too small");
    if (mode == QPSK_MODE_DEMODULATE && (!bits || !n_bits)) return fail(QPSK_ERR_ARGUMENT_NULL, "bits / n_bits required");
    if (mode == QPSK_MODE_CONSTELLATION && (!syms || !n_syms))
        return fail(QPSK_ERR_ARGUMENT_NULL, "syms / n_syms required");
    const int64_t max_sym = qpsk_demod_max_symbols(g->shards[0].h, n_call);
    if (bits && bits_stride_bytes < (2 * max_sym + 7) / 8)
        return fail(QPSK_ERR_ARGUMENT, "bits_stride_bytes smaller than 2*max_symbols/8");
    if (syms && syms_stride_floats < 2 * max_sym)
        return fail(QPSK_ERR_ARGUMENT, "syms_stride_floats smaller than 2*max_symbols");
    if (mem == QPSK_MEM_DEVICE) {
        // one device pointer cannot address several GPUs' rows: device-memory
        // batches go to the shard handles (qpsk_demod_group_shard) directly
        for (const Shard &sh : g->shards)
            if (sh.device != g->shards[0].device)
                return fail(QPSK_ERR_ARGUMENT, "device-memory group calls need every shard on one device; "
                                               "call the shard handles (qpsk_demod_group_shard) instead");
    }
    return fan_out(g, [=](int k) {
        const Shard &sh = g->shards[k];
        const int64_t f = sh.first;
        int rc = qpsk_demod_process(sh.h, mode, iq ? iq + f * stride_floats : nullptr, stride_floats, n_samples,
                                    lengths ? lengths + f : nullptr, mem, bits ? bits + f * bits_stride_bytes : nullptr,
                                    bits_stride_bytes, n_bits ? n_bits + f : nullptr,
                                    syms ? syms + f * syms_stride_floats : nullptr, syms_stride_floats,
                                    n_syms ? n_syms + f : nullptr);
        // device-memory calls are stream-ordered per shard: the group joins
        if (rc == QPSK_OK && mem == QPSK_MEM_DEVICE) rc = qpsk::handle_sync(sh.h);
        return rc;
    });
}

int64_t qpsk_demod_group_state_bytes(const qpsk_demod_group *g, int32_t k) {
    if (!g || k < 0 || k >= static_cast<int32_t>(g->shards.size())) return 0;
    return qpsk_demod_state_bytes(g->shards[k].h);
}

int qpsk_demod_group_get_state(qpsk_demod_group *g, int32_t k, void *host_buf, int64_t buf_bytes) {
    if (!g) return fail(QPSK_ERR_ARGUMENT_NULL, "null group");
    if (k < 0 || k >= static_cast<int32_t>(g->shards.size())) return fail(QPSK_ERR_ARGUMENT, "no such shard");
    return qpsk_demod_get_state(g->shards[k].h, host_buf, buf_bytes);
}

int qpsk_demod_group_set_state(qpsk_demod_group *g, int32_t k, const void *host_buf, int64_t buf_bytes) {
    if (!g) return fail(QPSK_ERR_ARGUMENT_NULL, "null group");
    if (k < 0 || k >= static_cast<int32_t>(g->shards.size())) return fail(QPSK_ERR_ARGUMENT, "no such shard");
    return qpsk_demod_set_state(g->shards[k].h, host_buf, buf_bytes);
}

}  // extern "C"
