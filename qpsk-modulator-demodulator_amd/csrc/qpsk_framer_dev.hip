// qpsk_framer_dev.hip -- device-resident byte framer (DeModulateBytes,
// QPSKDeModulator.cs:169-259) and batched TSC search (:413-422), SURVEY.md §8f
// rank 1.
//
// One 256-thread workgroup per stream runs one DeModulateBytes step on the
// packed bit row process() left in HBM.  The reference walks the bits as a
// '0'/'1' string; here every stage is a data-parallel pass over the packed row:
//
//   start hunt   BitsToBytes(cand, off) + IndexOf for off = 0..7 (:187-200)
//                == the first bit position q of the marker's bit pattern with
//                the smallest q mod 8 (the offset loop runs first, the byte
//                index second); each thread scans 32 positions from one 64-bit
//                window and the 8 per-offset minima reduce in LDS
//   append       AppendBitsToRing (:108-129) == a funnel-shifted copy of the
//                bit row behind the packer's partial byte into the ring
//   end search   RingIndexOf from count - (appended + |end|) (:133-149, :246)
//   copy-out     RingCopyOut + ResetFramer (:151-167)
//
// Work per call is O(bits) with no serial walk, and the scans stop at the
// first match (the chunk holding it): on real traffic the start and end
// markers sit near the start of a call's bits, and a frame that closes in the
// call never writes its bytes to the ring (its payload is copied straight from
// the bits).  The framer moves ~2 bits per symbol of traffic, noise next to
// the demod chain's 8 B/sample.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstring>
#include <string>
#include <vector>

#include "qpsk_demod.h"

namespace qpsk {
int set_last_error(int code, const std::string &msg);
}

namespace {

constexpr int kFrThreads = 256;
constexpr int64_t kRefRing = 300000000;   // FrameBuffer = new byte[300_000_000] (:58)

struct FrState {            // one reference instance's framer fields (:59-70)
    int32_t in_frame;       // _inFrame
    int32_t locked_off;     // _lockedBitOffset
    int32_t pack_byte;      // _packByte
    int32_t pack_bits;      // _packBits
    int64_t count;          // _rbCount (head == count: RingClear zeroes both, nothing pops)
    int64_t carry_bits;     // _searchCarryBits.Length (bits kept packed, MSB-first)
};

struct FrArgs {
    const uint8_t *bits;
    int64_t bits_stride;
    const int64_t *bit_offset;
    const int64_t *n_bits;
    uint8_t *payload;
    int64_t payload_stride;
    int64_t *n_payload;
    FrState *st;
    uint8_t *carry;         // [S][carry_stride]
    int64_t carry_stride;
    uint8_t *scratch;       // [S][scr_stride]  candidate bits of a start hunt
    int64_t scr_stride;
    uint8_t *ring;          // [S][ring_cap]
    int64_t ring_cap;
    const uint8_t *start;   // markers (device)
    int32_t ns;
    const uint8_t *end;
    int32_t ne;
};

__device__ inline uint32_t bit_at(const uint8_t *row, int64_t p) {
    return (row[p >> 3] >> (7 - (p & 7))) & 1u;
}

// 8 bits at bit position p (p + 8 <= valid bits of row).
__device__ inline uint32_t bits8(const uint8_t *row, int64_t p) {
    const int64_t b = p >> 3;
    const int sh = static_cast<int>(p & 7);
    uint32_t v = static_cast<uint32_t>(row[b]) << 8;
    if (sh) v |= row[b + 1];
    return (v >> (8 - sh)) & 0xffu;
}

// 64 bits from byte b on (MSB-first), bytes at or past nbytes read as 0.
__device__ inline uint64_t load_be64(const uint8_t *row, int64_t b, int64_t nbytes) {
    uint64_t w = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) w = (w << 8) | (b + i < nbytes ? row[b + i] : 0u);
    return w;
}

// 64 bits from byte b on (MSB-first) of a 4-byte aligned buffer holding at
// least b + 8 bytes: two dword loads and a byte swap instead of 8 byte loads
__device__ inline uint64_t load_be64_aligned(const uint8_t *buf, int64_t b) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(buf + b);
    return (static_cast<uint64_t>(__builtin_bswap32(w[0])) << 32) | __builtin_bswap32(w[1]);
}

// 64 bits from byte b on (MSB-first) of a row at any alignment whose valid
// bytes end at nbytes (bytes past it read as 0).  Windows whose 12 bytes lie
// inside the row take three aligned dword loads and a funnel shift; the rest
// (the row's last bytes) go byte by byte, so nothing past the row is read.
__device__ inline uint64_t load_be64_any(const uint8_t *row, int64_t b, int64_t nbytes) {
    const uintptr_t addr = reinterpret_cast<uintptr_t>(row + b);
    const int m = static_cast<int>(addr & 3);
    if (b + 12 <= nbytes) {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(addr - m);
        const uint64_t lo = static_cast<uint64_t>(w[0]) | (static_cast<uint64_t>(w[1]) << 32);
        const uint64_t hi = w[2];
        // little-endian bytes m .. m+7 of the 12 loaded
        const uint64_t v = m ? (lo >> (8 * m)) | (hi << (64 - 8 * m)) : lo;
        return __builtin_bswap64(v);
    }
    return load_be64(row, b, nbytes);
}

// The candidate bit string of a hunt: carry bits, then the row from bit off0.
struct Cand {
    const uint8_t *carry;
    int64_t ncarry;
    const uint8_t *row;
    int64_t off0;
    __device__ uint32_t bit(int64_t q) const {
        return q < ncarry ? bit_at(carry, q) : bit_at(row, off0 + q - ncarry);
    }
    // bits [q, q + 8) (q + 8 <= the string's length)
    __device__ uint32_t bits8_at(int64_t q) const {
        if (q >= ncarry) return bits8(row, off0 + q - ncarry);
        if (q + 8 <= ncarry) return bits8(carry, q);
        uint32_t v = 0;
        for (int i = 0; i < 8; ++i) v = (v << 1) | bit(q + i);
        return v;
    }
    // byte j of the candidate string (bits 8j..8j+7, zero past n)
    __device__ uint32_t byte(int64_t j, int64_t n) const {
        const int64_t q = 8 * j;
        if (q >= ncarry && q + 8 <= n) return bits8(row, off0 + q - ncarry);
        if (q + 8 <= ncarry) return carry[j];
        uint32_t v = 0;
        for (int i = 0; i < 8; ++i) v = (v << 1) | (q + i < n ? bit(q + i) : 0u);
        return v;
    }
};

__device__ void reset_state(FrState &s) {   // ResetFramer (:159-167)
    s.in_frame = 0;
    s.locked_off = -1;
    s.pack_byte = 0;
    s.pack_bits = 0;
    s.count = 0;
    s.carry_bits = 0;
}

// Positions a hunt / search chunk covers before the workgroup looks at its
// result: the reference's scans stop at the first match (IndexOf,
// RingIndexOf), and on real traffic that sits near the start of the row, so
// the chunks run in ascending position order and stop as soon as the answer
// cannot change.  (Until round 6 every position of the row was scanned and
// the whole row copied into the candidate scratch and the ring first.)
constexpr int kHuntWindows = kFrThreads;        // 32 positions each: 1 KB of candidate bits
constexpr int kEndPerThread = 8;                // ring positions per thread and chunk

__global__ void __launch_bounds__(kFrThreads) framer_push_kernel(FrArgs a) {
    __shared__ unsigned long long best[8];
    __shared__ unsigned long long best_end;
    const int s = blockIdx.x;
    const int tid = threadIdx.x;
    const int64_t off0 = a.bit_offset ? a.bit_offset[s] : 0;
    const int64_t nb = a.n_bits[s] - off0;
    if (tid == 0) a.n_payload[s] = 0;
    if (off0 < 0 || nb <= 0) return;                       // rxBits empty (:179-180)

    const uint8_t *row = a.bits + s * a.bits_stride;
    uint8_t *ring = a.ring + s * a.ring_cap;
    FrState st = a.st[s];
    __syncthreads();                       // every wave holds st before thread 0 may rewrite it

    // the bytes this call appends to the ring, as a function (materialised only
    // when the frame stays open past this call): case A = candidate bits from
    // the end of the start marker, case B = the packer's partial byte + rxBits
    bool entering = false;                 // case A (the frame opens in this call)
    Cand src{nullptr, 0, row, off0};
    int64_t mend = 0;                      // case A: first candidate bit after the start marker
    const int P = st.pack_bits;            // case B
    const uint32_t pack_byte = static_cast<uint32_t>(st.pack_byte);
    int64_t produced = 0;
    int rem = 0;

    if (!st.in_frame) {
        // ---- 1) start hunt over carry + rxBits (:183-236) ----
        // BitsToBytes(cand, off) + IndexOf for off = 0..7 == the first bit
        // position q of the marker pattern with the smallest q mod 8; every
        // thread tests 32 positions of one 64-bit window per chunk
        uint8_t *carry = a.carry + s * a.carry_stride;
        uint8_t *cand = a.scratch + s * a.scr_stride;
        src.carry = carry;
        src.ncarry = st.carry_bits;
        const int64_t nc = st.carry_bits + nb;
        const int64_t ncb = (nc + 7) >> 3;
        const int64_t pad_end = ncb + 8;                 // zero bytes behind the string (scratch slack)
        if (tid < 8) best[tid] = ULLONG_MAX;
        const int64_t limit = nc - 8 * static_cast<int64_t>(a.ns);   // last start position
        const uint32_t m0 = a.start[0];
        int64_t mat = 0;                                 // candidate bytes [0, mat) are in the scratch
        for (int64_t w0 = 0; 32 * w0 <= limit; w0 += kHuntWindows) {
            // the chunk's windows read bytes < 4 (w0 + kHuntWindows) + 8, the
            // marker checks up to ns + 1 bytes beyond
            int64_t need = 4 * (w0 + kHuntWindows) + 8 + a.ns + 1;
            need = need < pad_end ? need : pad_end;
            for (int64_t j = mat + tid; j < need; j += kFrThreads)
                cand[j] = static_cast<uint8_t>(j < ncb ? src.byte(j, nc) : 0u);
            mat = need > mat ? need : mat;
            __syncthreads();
            const int64_t w = w0 + tid;
            if (32 * w <= limit) {
                const uint64_t win = load_be64_aligned(cand, 4 * w);
                const int jmax = static_cast<int>(limit - 32 * w < 31 ? limit - 32 * w : 31);
                for (int j = 0; j <= jmax; ++j) {
                    if (((win >> (56 - j)) & 0xffu) != m0) continue;
                    const int64_t q = 32 * w + j;
                    int k = 1;
                    while (k < a.ns && bits8(cand, q + 8 * k) == a.start[k]) ++k;
                    if (k == a.ns) atomicMin(&best[j & 7], static_cast<unsigned long long>(q));
                }
            }
            __syncthreads();
            // offset 0 matched: no later chunk can hold a smaller offset-0
            // position, and offset 0 wins over every other offset
            if (best[0] != ULLONG_MAX) break;
        }
        int64_t q = -1;
        int off = -1;
        for (int o = 0; o < 8; ++o)
            if (best[o] != ULLONG_MAX) { q = static_cast<int64_t>(best[o]); off = o; break; }

        if (q < 0) {
            // no start: keep min(|cand|, 8|start|+7) tail bits (:233-235),
            // copied from the scratch (the carry is rewritten in place)
            for (int64_t j = mat + tid; j < pad_end; j += kFrThreads)
                cand[j] = static_cast<uint8_t>(j < ncb ? src.byte(j, nc) : 0u);
            __syncthreads();
            const int64_t keep = nc < 8 * static_cast<int64_t>(a.ns) + 7 ? nc : 8 * static_cast<int64_t>(a.ns) + 7;
            const int64_t base = nc - keep;
            for (int64_t j = tid; j < (keep + 7) >> 3; j += kFrThreads) {
                const int64_t p = base + 8 * j;
                uint32_t v;
                if (p + 8 <= nc) v = bits8(cand, p);
                else {
                    v = 0;
                    for (int i = 0; i < 8; ++i) v = (v << 1) | (p + i < nc ? bit_at(cand, p + i) : 0u);
                }
                carry[j] = static_cast<uint8_t>(v);
            }
            if (tid == 0) {
                st.carry_bits = keep;
                a.st[s] = st;
            }
            return;
        }
        // enter the frame: ring cleared, payload = cand bits after the marker (:203-214)
        mend = q + 8 * static_cast<int64_t>(a.ns);
        const int64_t len = nc - mend;
        produced = len >> 3;
        if (produced > a.ring_cap) {                         // overflow -> drop + resync (:215-220)
            if (tid == 0) {
                reset_state(st);
                a.st[s] = st;
            }
            return;
        }
        entering = true;
        st.in_frame = 1;
        st.locked_off = off;
        rem = static_cast<int>(len & 7);
        uint32_t pb = 0;
        for (int r = 0; r < rem; ++r) pb = (pb << 1) | src.bit(mend + 8 * produced + r);
        st.pack_byte = static_cast<int32_t>(pb);
        st.pack_bits = rem;
        st.count = 0;                                        // the ring restarts (RingClear)
    } else {
        // ---- 2) inside a frame: pack rxBits behind the partial byte (:238-246) ----
        const int64_t total = P + nb;
        produced = total >> 3;
        if (st.count + produced > a.ring_cap) {
            if (tid == 0) {
                reset_state(st);
                a.st[s] = st;
            }
            return;
        }
        // leftover bits: W[8*produced, total) of W = pack prefix + rxBits
        rem = static_cast<int>(total & 7);
        uint32_t pb = 0;
        for (int r = 0; r < rem; ++r) {
            const int64_t w = 8 * produced + r;
            pb = (pb << 1) | (w < P ? (pack_byte >> (P - 1 - w)) & 1u : bit_at(row, off0 + w - P));
        }
        st.pack_byte = static_cast<int32_t>(pb);
        st.pack_bits = rem;
    }
    const int64_t old_count = st.count;
    const int64_t count = old_count + produced;
    // byte j of this call's appended bytes (j < produced)
    auto newbyte = [&](int64_t j) -> uint32_t {
        if (entering) return src.bits8_at(mend + 8 * j);
        if (j == 0 && P > 0) {
            uint32_t v = pack_byte;
            for (int i = 0; i < 8 - P; ++i) v = (v << 1) | bit_at(row, off0 + i);
            return v & 0xffu;
        }
        return bits8(row, off0 + 8 * j - P);
    };
    // ring byte i after the append (i < count), without writing the ring
    auto ring_byte = [&](int64_t i) -> uint32_t { return i < old_count ? ring[i] : newbyte(i - old_count); };

    // ---- 3) end search: RingIndexOf from count - (appended + |end|) (:133-149, :246)
    const int64_t from = count - (produced + a.ne) > 0 ? count - (produced + a.ne) : 0;
    const int64_t last = count - a.ne;                       // last start position of the end marker
    if (tid == 0) best_end = ULLONG_MAX;
    __syncthreads();
    const uint32_t e0 = a.end[0];
    for (int64_t c0 = from; c0 <= last; c0 += kFrThreads * kEndPerThread) {
#pragma unroll
        for (int k = 0; k < kEndPerThread; ++k) {
            const int64_t i = c0 + k * kFrThreads + tid;
            if (i > last || ring_byte(i) != e0) continue;
            int m = 1;
            while (m < a.ne && ring_byte(i + m) == a.end[m]) ++m;
            if (m == a.ne) atomicMin(&best_end, static_cast<unsigned long long>(i));
        }
        __syncthreads();
        if (best_end != ULLONG_MAX) break;                   // the first occurrence is in this chunk
    }
    const int64_t end_at = best_end == ULLONG_MAX ? -1 : static_cast<int64_t>(best_end);
    if (end_at >= 0) {                                       // RingCopyOut + ResetFramer (:223-226)
        // the frame closes: its payload comes straight from the ring and this
        // call's bits; the appended bytes never need to be stored
        uint8_t *out = a.payload ? a.payload + s * a.payload_stride : nullptr;
        const int64_t n = end_at < a.payload_stride ? end_at : a.payload_stride;
        if (out)
            for (int64_t i = tid; i < n; i += kFrThreads) out[i] = static_cast<uint8_t>(ring_byte(i));
        if (tid == 0) {
            a.n_payload[s] = end_at;
            reset_state(st);
            a.st[s] = st;
        }
        return;
    }
    // the frame stays open: the appended bytes go into the ring (AppendBitsToRing)
    for (int64_t j = tid; j < produced; j += kFrThreads) ring[old_count + j] = static_cast<uint8_t>(newbyte(j));
    if (tid == 0) {
        st.count = count;
        a.st[s] = st;
    }
}

// Pattern bits ride by value in the kernel arguments up to 4096 bits (the
// reference's TSC is 64, testAtDataLevel.cs:20-22); longer ones in a buffer.
struct TscPat {
    uint8_t b[512];
};

// rx.IndexOf(tsc, Ordinal) per stream (:413-422).  Each thread tests 32
// positions against the first min(m, 32) pattern bits from one 64-bit window,
// the rest bit by bit; the minimum position reduces in LDS.  Chunks of
// kFrThreads windows run in ascending position order and the search stops
// after the chunk holding the first match.
__global__ void __launch_bounds__(kFrThreads)
tsc_find_kernel(const uint8_t *bits, int64_t stride, const int64_t *n_bits, TscPat small,
                const uint8_t *big, int32_t m, int64_t *offsets) {
    __shared__ unsigned long long best;
    const uint8_t *pat = big ? big : small.b;
    const int s = blockIdx.x;
    const uint8_t *row = bits + s * stride;
    const int64_t n = n_bits[s];
    const int64_t limit = n - m;
    const int64_t nbytes = (n + 7) >> 3;
    const int km = m < 32 ? m : 32;
    uint32_t key = 0;
    for (int i = 0; i < km; ++i) key = (key << 1) | bit_at(pat, i);
    const uint64_t kmask = km == 32 ? 0xffffffffull : ((1ull << km) - 1);
    if (threadIdx.x == 0) best = ULLONG_MAX;
    __syncthreads();
    for (int64_t w0 = 0; 32 * w0 <= limit; w0 += kFrThreads) {
        const int64_t w = w0 + threadIdx.x;
        if (32 * w <= limit) {
            const uint64_t win = load_be64_any(row, 4 * w, nbytes);
            const int jmax = static_cast<int>(limit - 32 * w < 31 ? limit - 32 * w : 31);
            // position j of the window matches the first km pattern bits
            auto full = [&](int j) -> bool {
                if (j > jmax || ((win >> (64 - km - j)) & kmask) != key) return false;
                const int64_t q = 32 * w + j;
                int k = km;
                while (k < m && bit_at(row, q + k) == bit_at(pat, k)) ++k;
                return k == m;
            };
            if (m >= 16) {
                // a 16-bit prefix filter on two positions per 32-bit word: the
                // word of bits [o, o + 32) holds the 16-bit values at o (high
                // half) and o + 16 (low half), so 16 funnel shifts cover the
                // window's 32 positions; a half equal to the prefix (haszero on
                // the XOR, false positives possible, never false negatives) is
                // checked in full.  ~5 ops per two positions instead of ~6 per one
                const uint32_t k16 = key >> (km - 16);
                const uint32_t kk = (k16 << 16) | k16;
                const uint32_t whi = static_cast<uint32_t>(win >> 32), wlo = static_cast<uint32_t>(win);
                int first = 64;
#pragma unroll
                for (int o = 0; o < 16; ++o) {
                    const uint32_t x = o ? (whi << o) | (wlo >> (32 - o)) : whi;
                    const uint32_t z = x ^ kk;
                    const uint32_t hz = (z - 0x00010001u) & ~z & 0x80008000u;
                    if (__builtin_expect(hz != 0, 0)) {
                        if ((hz & 0x80000000u) && o < first && full(o)) first = o;
                        if ((hz & 0x00008000u) && o + 16 < first && full(o + 16)) first = o + 16;
                    }
                }
                if (first < 64) atomicMin(&best, static_cast<unsigned long long>(32 * w + first));
            } else {
                for (int j = 0; j <= jmax; ++j) {
                    if (full(j)) {
                        atomicMin(&best, static_cast<unsigned long long>(32 * w + j));
                        break;                               // later j of this window are larger
                    }
                }
            }
        }
        __syncthreads();
        if (best != ULLONG_MAX) break;                       // no later chunk holds a smaller one
    }
    if (threadIdx.x == 0) offsets[s] = best == ULLONG_MAX ? -1 : static_cast<int64_t>(best) + m;
}

int fail(int code, const std::string &msg) { return qpsk::set_last_error(code, msg); }

#define FR_TRY(expr)                                                                   \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return fail(QPSK_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

}  // namespace

struct qpsk_framer_dev {
    int32_t n_streams = 0;
    int32_t device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    FrState *st = nullptr;
    uint8_t *carry = nullptr;
    int64_t carry_stride = 0;
    uint8_t *scratch = nullptr;
    int64_t scr_stride = 0;
    uint8_t *ring = nullptr;
    int64_t ring_cap = kRefRing;
    uint8_t *markers = nullptr;      // start bytes then end bytes
    int64_t markers_cap = 0;
    int32_t ns = 0, ne = 0;

    ~qpsk_framer_dev() {
        if (stream) hipStreamSynchronize(stream);
        hipFree(st);
        hipFree(carry);
        hipFree(scratch);
        hipFree(ring);
        hipFree(markers);
        if (own_stream && stream) hipStreamDestroy(stream);
    }
};

namespace {
// Markers go to device memory after the stream drained; a longer start marker
// widens every stream's carry row (8|start|+7 bits), keeping the bits held.
int load_markers(qpsk_framer_dev *f, const uint8_t *start, int32_t ns, const uint8_t *end, int32_t ne) {
    if (!start || !end) return fail(QPSK_ERR_ARGUMENT_NULL, "marker is null");
    if (ns <= 0) return fail(QPSK_ERR_ARGUMENT, "startMarker cannot be empty.");   // :174
    if (ne <= 0) return fail(QPSK_ERR_ARGUMENT, "endMarker cannot be empty.");     // :175
    FR_TRY(hipSetDevice(f->device));
    if (f->stream) FR_TRY(hipStreamSynchronize(f->stream));
    if (static_cast<int64_t>(ns) + ne > f->markers_cap) {
        hipFree(f->markers);
        f->markers = nullptr;
        f->markers_cap = static_cast<int64_t>(ns) + ne;
        FR_TRY(hipMalloc(reinterpret_cast<void **>(&f->markers), f->markers_cap));
    }
    std::vector<uint8_t> m(start, start + ns);
    m.insert(m.end(), end, end + ne);
    FR_TRY(hipMemcpy(f->markers, m.data(), m.size(), hipMemcpyHostToDevice));
    const int64_t need = ((static_cast<int64_t>(ns) + 1 + 15) / 16) * 16;
    if (need > f->carry_stride) {
        uint8_t *c = nullptr;
        FR_TRY(hipMalloc(reinterpret_cast<void **>(&c), need * f->n_streams));
        FR_TRY(hipMemset(c, 0, need * f->n_streams));
        if (f->carry)
            FR_TRY(hipMemcpy2D(c, need, f->carry, f->carry_stride, f->carry_stride, f->n_streams,
                               hipMemcpyDeviceToDevice));
        hipFree(f->carry);
        f->carry = c;
        f->carry_stride = need;
    }
    f->ns = ns;
    f->ne = ne;
    return QPSK_OK;
}
}  // namespace

extern "C" {

int qpsk_framer_dev_create(int32_t n_streams, const uint8_t *start_marker, int32_t n_start,
                           const uint8_t *end_marker, int32_t n_end, int64_t ring_capacity,
                           int32_t device, qpsk_framer_dev **out) {
    if (!out) return fail(QPSK_ERR_ARGUMENT_NULL, "out is null");
    *out = nullptr;
    if (n_streams <= 0) return fail(QPSK_ERR_ARGUMENT, "n_streams must be positive");
    auto *f = new qpsk_framer_dev();
    f->n_streams = n_streams;
    f->device = device;
    if (ring_capacity > 0) f->ring_cap = ring_capacity;
    int rc = load_markers(f, start_marker, n_start, end_marker, n_end);
    if (rc != QPSK_OK) {
        delete f;
        return rc;
    }
    hipError_t e = hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking);
    if (e == hipSuccess) {
        f->own_stream = true;
        e = hipMalloc(reinterpret_cast<void **>(&f->ring), f->ring_cap * n_streams);
    }
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&f->st), sizeof(FrState) * n_streams);
    if (e == hipSuccess) {
        std::vector<FrState> init(n_streams, FrState{0, -1, 0, 0, 0, 0});
        e = hipMemcpy(f->st, init.data(), sizeof(FrState) * n_streams, hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
        delete f;
        return fail(QPSK_ERR_DEVICE, std::string("framer allocation: ") + hipGetErrorString(e));
    }
    *out = f;
    return QPSK_OK;
}

int qpsk_framer_dev_destroy(qpsk_framer_dev *f) {
    delete f;
    return QPSK_OK;
}

int qpsk_framer_dev_set_stream(qpsk_framer_dev *f, void *hip_stream) {
    if (!f) return fail(QPSK_ERR_ARGUMENT_NULL, "null framer");
    FR_TRY(hipSetDevice(f->device));
    FR_TRY(hipStreamSynchronize(f->stream));
    if (hip_stream) {
        if (f->own_stream) hipStreamDestroy(f->stream);
        f->stream = static_cast<hipStream_t>(hip_stream);
        f->own_stream = false;
    } else if (!f->own_stream) {
        FR_TRY(hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking));
        f->own_stream = true;
    }
    return QPSK_OK;
}

int qpsk_framer_dev_set_markers(qpsk_framer_dev *f, const uint8_t *start_marker, int32_t n_start,
                                const uint8_t *end_marker, int32_t n_end) {
    if (!f) return fail(QPSK_ERR_ARGUMENT_NULL, "null framer");
    return load_markers(f, start_marker, n_start, end_marker, n_end);
}

int qpsk_framer_dev_push(qpsk_framer_dev *f, const uint8_t *bits, int64_t bits_stride_bytes,
                         const int64_t *bit_offset, const int64_t *n_bits, uint8_t *payload,
                         int64_t payload_stride, int64_t *n_payload) {
    if (!f || !bits || !n_bits || !n_payload) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    if (bits_stride_bytes <= 0 || payload_stride < 0) return fail(QPSK_ERR_ARGUMENT, "bad stride");
    FR_TRY(hipSetDevice(f->device));
    // candidate row: carry (<= carry_stride bytes) + one row of bits, 8 B slack
    const int64_t need = ((f->carry_stride + bits_stride_bytes + 8 + 15) / 16) * 16;
    if (need > f->scr_stride) {
        FR_TRY(hipStreamSynchronize(f->stream));
        hipFree(f->scratch);
        f->scratch = nullptr;
        f->scr_stride = 0;
        FR_TRY(hipMalloc(reinterpret_cast<void **>(&f->scratch), need * f->n_streams));
        f->scr_stride = need;
    }
    FrArgs a;
    a.bits = bits;
    a.bits_stride = bits_stride_bytes;
    a.bit_offset = bit_offset;
    a.n_bits = n_bits;
    a.payload = payload_stride > 0 ? payload : nullptr;
    a.payload_stride = payload_stride;
    a.n_payload = n_payload;
    a.st = f->st;
    a.carry = f->carry;
    a.carry_stride = f->carry_stride;
    a.scratch = f->scratch;
    a.scr_stride = f->scr_stride;
    a.ring = f->ring;
    a.ring_cap = f->ring_cap;
    a.start = f->markers;
    a.ns = f->ns;
    a.end = f->markers + f->ns;
    a.ne = f->ne;
    hipLaunchKernelGGL(framer_push_kernel, dim3(f->n_streams), dim3(kFrThreads), 0, f->stream, a);
    FR_TRY(hipGetLastError());
    return QPSK_OK;
}

int qpsk_framer_dev_status(const qpsk_framer_dev *f, int32_t *in_frame, int64_t *ring_count,
                           int64_t *carry_bits) {
    if (!f) return fail(QPSK_ERR_ARGUMENT_NULL, "null framer");
    FR_TRY(hipSetDevice(f->device));
    FR_TRY(hipStreamSynchronize(f->stream));
    std::vector<FrState> h(f->n_streams);
    FR_TRY(hipMemcpy(h.data(), f->st, sizeof(FrState) * f->n_streams, hipMemcpyDeviceToHost));
    for (int32_t s = 0; s < f->n_streams; ++s) {
        if (in_frame) in_frame[s] = h[s].in_frame;
        if (ring_count) ring_count[s] = h[s].count;
        if (carry_bits) carry_bits[s] = h[s].carry_bits;
    }
    return QPSK_OK;
}

int qpsk_tsc_find_device(const uint8_t *bits, int64_t bits_stride_bytes, const int64_t *n_bits,
                         int32_t n_streams, const char *tsc, int64_t *offsets, void *hip_stream) {
    if (!offsets || !n_bits) return fail(QPSK_ERR_ARGUMENT_NULL, "null argument");
    if (n_streams <= 0) return QPSK_OK;
    hipStream_t stream = static_cast<hipStream_t>(hip_stream);
    const int64_t m = tsc ? static_cast<int64_t>(std::strlen(tsc)) : 0;
    bool blank = true;                                       // string.IsNullOrWhiteSpace (:21)
    bool binary = true;
    for (int64_t i = 0; i < m; ++i) {
        if (!std::strchr(" \t\r\n\v\f", tsc[i])) blank = false;
        if (tsc[i] != '0' && tsc[i] != '1') binary = false;
    }
    if (blank) {                                             // no TSC: payload = every bit
        FR_TRY(hipMemsetAsync(offsets, 0, sizeof(int64_t) * n_streams, stream));
        return QPSK_OK;
    }
    if (!binary || m > INT32_MAX) {                          // '0'/'1' rows never match other chars
        FR_TRY(hipMemsetAsync(offsets, 0xff, sizeof(int64_t) * n_streams, stream));
        return QPSK_OK;
    }
    if (!bits) return fail(QPSK_ERR_ARGUMENT_NULL, "bits is null");
    if (bits_stride_bytes <= 0) return fail(QPSK_ERR_ARGUMENT, "bad stride");
    std::vector<uint8_t> packed((m + 7) / 8, 0);
    for (int64_t i = 0; i < m; ++i)
        if (tsc[i] == '1') packed[i >> 3] |= static_cast<uint8_t>(0x80u >> (i & 7));
    TscPat small{};
    uint8_t *big = nullptr;
    if (packed.size() <= sizeof(small.b)) {
        std::memcpy(small.b, packed.data(), packed.size());
    } else {                                                 // rare: stream-ordered buffer
        FR_TRY(hipMallocAsync(reinterpret_cast<void **>(&big), packed.size(), stream));
        FR_TRY(hipMemcpyAsync(big, packed.data(), packed.size(), hipMemcpyHostToDevice, stream));
    }
    hipLaunchKernelGGL(tsc_find_kernel, dim3(n_streams), dim3(kFrThreads), 0, stream, bits,
                       bits_stride_bytes, n_bits, small, static_cast<const uint8_t *>(big),
                       static_cast<int32_t>(m), offsets);
    FR_TRY(hipGetLastError());
    if (big) {
        FR_TRY(hipFreeAsync(big, stream));
        FR_TRY(hipStreamSynchronize(stream));               // pageable source outlives the copy
    }
    return QPSK_OK;
}

}  // extern "C"
