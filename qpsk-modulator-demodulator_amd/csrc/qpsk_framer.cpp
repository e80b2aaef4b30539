// qpsk_framer.cpp -- batched byte framer (DeModulateBytes, QPSKDeModulator.cs:169-259)
// and TSC search (QPSKDeModulator.cs:413-422), host side.
//
// One framer per stream reproduces the reference state machine exactly: start
// marker hunt at bit offsets 0..7 over carry + new bits (BitPacker.BitsToBytes /
// IndexOf, HelperFunctions.cs:32-70), MSB-first packing into a bounded ring,
// end-marker search from count - (appended + |end|), overflow -> drop + resync.
// The reference's 300 MB ring (QPSKDeModulator.cs:58) becomes a per-stream
// capacity parameter with the same overflow semantics.
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "qpsk_demod.h"

namespace {
thread_local std::string g_framer_err;

struct StreamFramer {
    std::vector<uint8_t> ring;     // payload bytes (ring contents in order)
    bool in_frame = false;
    std::vector<uint8_t> carry;    // _searchCarryBits as 0/1 values
    int locked_off = -1;
    uint8_t pack_byte = 0;
    int pack_bits = 0;

    void reset() {   // ResetFramer (:159-167)
        in_frame = false;
        locked_off = -1;
        carry.clear();
        ring.clear();
        pack_byte = 0;
        pack_bits = 0;
    }
};

// AppendBitsToRing (:108-129): -1 on overflow
int64_t append_bits(StreamFramer &f, const uint8_t *b, int64_t n, int64_t cap) {
    int64_t produced = 0;
    for (int64_t i = 0; i < n; ++i) {
        f.pack_byte = static_cast<uint8_t>((f.pack_byte << 1) | (b[i] ? 1 : 0));
        if (++f.pack_bits == 8) {
            if (static_cast<int64_t>(f.ring.size()) >= cap) return -1;
            f.ring.push_back(f.pack_byte);
            ++produced;
            f.pack_bits = 0;
            f.pack_byte = 0;
        }
    }
    return produced;
}

// RingIndexOf (:133-149)
int64_t ring_index_of(const StreamFramer &f, const uint8_t *pat, int64_t np, int64_t from) {
    if (np == 0) return 0;
    const int64_t cnt = static_cast<int64_t>(f.ring.size());
    if (cnt < np) return -1;
    for (int64_t i = std::max<int64_t>(0, from); i <= cnt - np; ++i)
        if (std::memcmp(f.ring.data() + i, pat, np) == 0) return i;
    return -1;
}

inline uint8_t bit_at(const uint8_t *packed, int64_t i) {
    return static_cast<uint8_t>((packed[i >> 3] >> (7 - (i & 7))) & 1);
}
}  // namespace

struct qpsk_framer {
    std::vector<StreamFramer> st;
    std::vector<uint8_t> start, end;
    int64_t ring_cap = 300000000;
};

extern "C" {

int qpsk_framer_create(int32_t n_streams, const uint8_t *start_marker, int32_t n_start,
                       const uint8_t *end_marker, int32_t n_end, int64_t ring_capacity,
                       qpsk_framer **out) {
    if (!out) return QPSK_ERR_ARGUMENT_NULL;
    *out = nullptr;
    if (n_streams <= 0) return QPSK_ERR_ARGUMENT;
    if (n_start <= 0 || !start_marker) return QPSK_ERR_ARGUMENT;   // :174
    if (n_end <= 0 || !end_marker) return QPSK_ERR_ARGUMENT;       // :175
    auto *f = new qpsk_framer();
    f->st.resize(n_streams);
    f->start.assign(start_marker, start_marker + n_start);
    f->end.assign(end_marker, end_marker + n_end);
    if (ring_capacity > 0) f->ring_cap = ring_capacity;
    *out = f;
    return QPSK_OK;
}

int qpsk_framer_destroy(qpsk_framer *f) {
    delete f;
    return QPSK_OK;
}

int qpsk_framer_set_markers(qpsk_framer *f, const uint8_t *start_marker, int32_t n_start,
                            const uint8_t *end_marker, int32_t n_end) {
    if (!f) return QPSK_ERR_ARGUMENT_NULL;
    if (n_start <= 0 || !start_marker || n_end <= 0 || !end_marker) return QPSK_ERR_ARGUMENT;
    f->start.assign(start_marker, start_marker + n_start);
    f->end.assign(end_marker, end_marker + n_end);
    return QPSK_OK;
}

int qpsk_framer_push(qpsk_framer *f, const uint8_t *bits, int64_t bits_stride_bytes,
                     const int64_t *bit_offset, const int64_t *n_bits, uint8_t *payload,
                     int64_t payload_stride, int64_t *n_payload) {
    if (!f || !bits || !n_bits || !n_payload) return QPSK_ERR_ARGUMENT_NULL;
    const int64_t ns = static_cast<int64_t>(f->start.size());
    const int64_t ne = static_cast<int64_t>(f->end.size());
    std::vector<uint8_t> rx, cand, bytes;
    for (size_t s = 0; s < f->st.size(); ++s) {
        StreamFramer &F = f->st[s];
        n_payload[s] = 0;
        const int64_t off0 = bit_offset ? bit_offset[s] : 0;
        const int64_t nb = n_bits[s] - off0;
        if (off0 < 0 || nb <= 0) continue;                  // empty rxBits (:179-180)
        const uint8_t *row = bits + s * bits_stride_bytes;
        rx.resize(nb);
        for (int64_t i = 0; i < nb; ++i) rx[i] = bit_at(row, off0 + i);
        auto emit = [&](int64_t len) {
            const int64_t n = std::min<int64_t>(len, payload_stride);
            if (payload && n > 0) std::memcpy(payload + s * payload_stride, F.ring.data(), n);
            n_payload[s] = len;
        };
        if (!F.in_frame) {
            cand = F.carry;                                  // :185
            cand.insert(cand.end(), rx.begin(), rx.end());
            const int64_t nc = static_cast<int64_t>(cand.size());
            bool found = false;
            for (int off = 0; off < 8 && !found; ++off) {    // :187-230
                const int64_t usable = nc - off;
                if (usable < 8) continue;
                const int64_t nbytes = usable / 8;
                bytes.assign(nbytes, 0);
                for (int64_t i = 0; i < nbytes; ++i) {
                    uint8_t v = 0;
                    for (int j = 0; j < 8; ++j) v = static_cast<uint8_t>((v << 1) | cand[off + 8 * i + j]);
                    bytes[i] = v;
                }
                int64_t pos = -1;
                if (ns <= nbytes)
                    for (int64_t i = 0; i <= nbytes - ns; ++i)
                        if (std::memcmp(bytes.data() + i, f->start.data(), ns) == 0) { pos = i; break; }
                if (pos < 0) continue;
                const int64_t mend = off + 8 * (pos + ns);
                if (mend > nc) continue;
                found = true;
                F.in_frame = true;
                F.locked_off = off;
                F.ring.clear();
                F.pack_byte = 0;
                F.pack_bits = 0;
                const int64_t appended = append_bits(F, cand.data() + mend, nc - mend, f->ring_cap);
                if (appended < 0) { F.reset(); break; }
                const int64_t end_at = ring_index_of(
                    F, f->end.data(), ne, std::max<int64_t>(0, static_cast<int64_t>(F.ring.size()) - (appended + ne)));
                if (end_at >= 0) {
                    emit(end_at);
                    F.reset();
                }
            }
            if (!found) {                                    // :233-235
                const int64_t keep = std::min<int64_t>(nc, ns * 8 + 7);
                F.carry.assign(cand.end() - keep, cand.end());
            }
            continue;
        }
        const int64_t appended = append_bits(F, rx.data(), nb, f->ring_cap);   // :240
        if (appended < 0) { F.reset(); continue; }
        const int64_t from = std::max<int64_t>(0, static_cast<int64_t>(F.ring.size()) - (appended + ne));
        const int64_t end_at = ring_index_of(F, f->end.data(), ne, from);
        if (end_at >= 0) {
            emit(end_at);
            F.reset();
        }
    }
    return QPSK_OK;
}

int64_t qpsk_tsc_find(const uint8_t *bits, int64_t n_bits, const char *tsc) {
    if (!tsc) return 0;
    const int64_t m = static_cast<int64_t>(std::strlen(tsc));
    bool blank = true;                                        // string.IsNullOrWhiteSpace (:21)
    for (int64_t i = 0; i < m; ++i)
        if (!std::strchr(" \t\r\n\v\f", tsc[i])) { blank = false; break; }
    if (blank) return 0;
    if (!bits) return -1;
    for (int64_t i = 0; i + m <= n_bits; ++i) {
        int64_t j = 0;
        for (; j < m; ++j) {
            const char c = bit_at(bits, i + j) ? '1' : '0';
            if (c != tsc[j]) break;
        }
        if (j == m) return i + m;
    }
    return -1;
}

}  // extern "C"
