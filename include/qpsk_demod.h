/*
 * qpsk_demod.h -- C ABI of the MI355X-native batched QPSK demodulation chain.
 *
 * This is the drop-in boundary for the reference's QPSKDeModulator C# class
 * (NustyFrozen/QPSK-Modulator-Demodulator, Modulation-Simulation/QPSKDeModulator.cs).
 * The reference has no FFI layer; its boundary *is* that public class.  A C#
 * host binds these entry points with [DllImport("qpsk_demod")] (see
 * INTEGRATION.md); one handle serves a batch of S independent streams, each of
 * which behaves exactly like one QPSKDeModulator instance.
 *
 * Conventions (QPSKDeModulator.cs:339-425):
 *  - input is interleaved float32 I,Q; every call continues the previous call's
 *    FIR / FLL / Mueller-Muller / Costas / differential-decode state;
 *  - an odd float count is QPSK_ERR_ARGUMENT (ArgumentException, :347-348);
 *  - a zero-length call returns no bits and leaves the state untouched (:350-351);
 *  - the caller owns every I/O buffer, the library owns device buffers and the
 *    per-stream state; a handle is not thread-safe (one caller thread per
 *    handle), distinct handles are independent.
 * Every function returns an int status: 0 = ok, < 0 = error, message in
 * qpsk_last_error().
 */
#ifndef QPSK_DEMOD_H
#define QPSK_DEMOD_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 3: multi-GPU group (qpsk_shard_streams, qpsk_demod_group_*); no change to
 *    existing entry points or the state blob.
 * 2: versioned state blob (header + length checked by set_state; 256-sample
 *    M&M carry), get_state / set_state take the buffer length and a non-const
 *    handle (they flush pipelined work), qpsk_pipeline_gate_enabled.
 * 1: rounds 1-3. */
#define QPSK_ABI_VERSION 3

/* status codes -> the C# exception each one replaces */
#define QPSK_OK 0
#define QPSK_ERR_ARGUMENT (-1)        /* ArgumentException (odd length, empty marker) */
#define QPSK_ERR_ARGUMENT_NULL (-2)   /* ArgumentNullException (QPSKDeModulator.cs:341,429) */
#define QPSK_ERR_OUT_OF_RANGE (-3)    /* ArgumentOutOfRangeException (Band-Edge Filter.cs:42-45) */
#define QPSK_ERR_DEVICE (-4)          /* HIP runtime failure */
#define QPSK_ERR_CAPACITY (-5)        /* an output row would have been truncated */
#define QPSK_ERR_STATE (-6)           /* loop state left the reference's defined behaviour
                                         (QPSK_STATUS_CARRY_OVERFLOW / _NONFINITE_TIMING), or a
                                         host ring used out of order */

/* status flags (qpsk_demod_status; a host-memory process() call returns the
 * matching error code when its own call raised one) */
#define QPSK_STATUS_CARRY_OVERFLOW 1u    /* symbol-sync queue kept > 256 samples: the queue
                                            holds <= 3 samples between calls at any sps, more
                                            only when the M&M stops on output capacity (sps
                                            below ~1); the reference keeps them all
                                            (MuellerMuller.cs:123-133) */
#define QPSK_STATUS_OUTPUT_TRUNCATED 2u  /* a bit / symbol row hit its capacity */
#define QPSK_STATUS_NONFINITE_TIMING 4u  /* a NaN/Inf sample reached the M&M timing loop: the
                                            reference's (int)Math.Floor(NaN) = 0 pins baseIndex
                                            at 0 (MuellerMuller.cs:113-115) and its outputs are
                                            no longer tracked */

/* where a pointer lives */
#define QPSK_MEM_HOST 0
#define QPSK_MEM_DEVICE 1

/* what one call produces */
#define QPSK_MODE_DEMODULATE 0        /* DeModulate: bits (+ optional symbols) */
#define QPSK_MODE_CONSTELLATION 1     /* deModulateConstellation: symbols only, diff state untouched */

/* Mirrors the QPSKDeModulator primary constructor 1:1 (QPSKDeModulator.cs:11-18)
 * plus the batch / device knobs. */
typedef struct qpsk_demod_params {
    int32_t sample_rate;            /* int SampleRate                                   */
    int32_t symbol_rate;            /* int SymbolRate                                   */
    float rrc_alpha;                /* float RrcAlpha = 0.9f                            */
    int32_t rrc_span;               /* int rrcSpan = 6                                  */
    double symbol_sync_bandwidth;   /* double SymbolSyncBandwith = 0.0001               */
    double costas_loop_bandwidth;   /* double CostasLoopBandwith = 120                  */
    double cfo_loop_bandwidth;      /* double CFOLoopBandwith = 0.0001f                 */
    int32_t differential;           /* bool differentialEncoding = true                 */
    int32_t enable_fll;             /* 0 = reference DeModulate (fll.Process disabled, :359) */
    int32_t vector_lanes;           /* Vector<float>.Count whose summation order the FIR
                                       reproduces: 8 (x64 AVX2, default), 4 (ARM64), 1 (no SIMD) */
    int32_t device;                 /* HIP device ordinal                               */
    int64_t max_samples_per_call;   /* complex samples per stream per internal chunk (device
                                       buffers), 1 .. 2^30; longer calls run as consecutive
                                       chunks with identical results */
    int32_t loop_variant;           /* symbol-loop kernel shape: 0 = auto,
                                       1 = 16 streams x 64-sample rounds, 2 = 32 x 64,
                                       3 = 16 x 128 (sps >= 2 only), 4 = 24 x 128 (sps >= 8
                                       only, else auto), 5 = retired (64 x 32,
                                       measured slower; runs as auto), 6 = 12 x 256,
                                       7 = 6 x 512 (both sps >= 8 only, else auto;
                                       32 busy lanes); results are
                                       identical */
    int32_t iq_balance;             /* 1 = IQ_Balancer.Process (IQ Balancer.cs:15-25) on every
                                       sample before the FLL / matched filter; 0 (default) =
                                       the reference DeModulate, which constructs the balancer
                                       (QPSKDeModulator.cs:38) but never calls it */
    int32_t costas_trig;            /* the Costas NCO's Math.Cos / Math.Sin (CostasLoopQpsk.cs:69-70):
                                       0 (default) = a portable table sincos within 1 ulp of
                                       glibc (bit-identical on ~98.7 % of arguments); 1 = glibc's
                                       own sin / cos restated exactly (what .NET calls on Linux
                                       x86-64; symbols bit-identical by construction, slower) */
    int32_t reserved[5];
} qpsk_demod_params;

typedef struct qpsk_demod qpsk_demod;

/* Fill defaults exactly as the C# optional parameters. */
void qpsk_demod_params_init(qpsk_demod_params *p, int32_t sample_rate, int32_t symbol_rate);

/* new QPSKDeModulator(...) x n_streams  (QPSKDeModulator.cs:11-56) */
int qpsk_demod_create(const qpsk_demod_params *p, int32_t n_streams, qpsk_demod **out);
int qpsk_demod_destroy(qpsk_demod *h);

/* Bind the handle to a caller-owned hipStream_t (NULL = library-owned stream). */
int qpsk_demod_set_stream(qpsk_demod *h, void *hip_stream);

/*
 * One DeModulate (mode 0) or deModulateConstellation (mode 1) call on every
 * stream of the batch  (QPSKDeModulator.cs:345-425 / :427-455).
 *
 * iq        [n_streams][stride_floats] float32, stream s holds
 *           2*len(s) floats, len(s) = lengths ? lengths[s] : n_samples
 * bits      [n_streams][bits_stride_bytes] raw demodulated bits of this call,
 *           packed MSB-first (BitPacker order, HelperFunctions.cs:14-29), before
 *           any TSC strip; may be NULL in mode 1
 * n_bits    [n_streams] bit counts (2 per symbol; the very first symbol of a
 *           differential stream yields none, :390-395)
 * syms      [n_streams][syms_stride_floats] rotated Costas output symbols
 *           (interleaved I,Q) or NULL
 * n_syms    [n_streams] symbol counts or NULL
 * mem       QPSK_MEM_HOST or QPSK_MEM_DEVICE for every pointer above
 * The call is synchronous for host pointers and stream-ordered for device ones.
 * Any length is accepted (QPSKDeModulator.cs:345-360 takes any span): a call
 * longer than max_samples_per_call runs as consecutive internal chunks whose
 * rows are concatenated, bit for bit what one call returns.  Host-memory calls
 * return QPSK_ERR_STATE / QPSK_ERR_CAPACITY when they raised a QPSK_STATUS_*
 * flag (outputs are still written); device-memory calls report them through
 * qpsk_demod_status.
 * Bytes of a bit row past the last bit (and floats of a symbol row past the
 * last symbol) are unspecified.  Device rows that are 4-byte aligned with
 * bits_stride_bytes % 4 == 0 (8-byte aligned, even syms_stride_floats for
 * symbols) are written in place by the loop kernel, whole 32-bit words up to
 * the row's last bit; other rows are filled from an internal buffer by a copy.
 */
int qpsk_demod_process(qpsk_demod *h, int32_t mode, const float *iq, int64_t stride_floats,
                       int64_t n_samples, const int64_t *lengths, int32_t mem, uint8_t *bits,
                       int64_t bits_stride_bytes, int64_t *n_bits, float *syms,
                       int64_t syms_stride_floats, int64_t *n_syms);

/*
 * Pipelined DeModulate calls (device memory only).  Same arguments, checks and
 * results as qpsk_demod_process(mem = QPSK_MEM_DEVICE); calls still apply to
 * every stream in order and carry the state exactly as synchronous calls do.
 * The difference is scheduling: each call is split into a front stage (FLL on:
 * the FLL; FLL off: the matched filter) and a back stage (the rest) on two
 * library streams, so call k+1's front stage runs while call k's symbol loop
 * runs.  A C# host feeding consecutive SDR buffers keeps the GPU busy this
 * way instead of waiting for each DeModulate to return.
 *  - iq is read after the work already queued on the handle's stream; it must
 *    stay unchanged until qpsk_demod_pipeline_wait has been called for it.
 *  - bits / n_bits / syms / n_syms are complete after qpsk_demod_pipeline_wait.
 *  - synchronous process(), get/set_state, set_stream and destroy first wait
 *    for every pipelined call.
 *  - Residency gate: call k+1's matched filter waits ON THE DEVICE (a
 *    one-wave kernel ahead of it on the front stream) until call k's
 *    symbol-loop workgroups hold their CUs, so the two always overlap in the
 *    same order.  The wait is bounded: after QPSK_GATE_TIMEOUT_MS (default
 *    2000 ms, read at create) the filter goes ahead and the timeout is counted
 *    (qpsk_demod_gate_timeouts); results never depend on the gate.  Under
 *    serialised dispatch the loop kernel could only start after the waiting
 *    filter, so every wait would run out: the gate is off when
 *    qpsk_pipeline_gate_enabled() says so:
 *    QPSK_PIPELINE_GATE=0, AMD_SERIALIZE_KERNEL or AMD_SERIALIZE_COPY != 0,
 *    HIP_LAUNCH_BLOCKING or CUDA_LAUNCH_BLOCKING != 0, rocprofv3 counter
 *    collection (ROCPROF_COUNTER_COLLECTION=1) or kernel serialisation
 *    (ROCPROFILER_KERNEL_SERIALIZATION), HSA_ENABLE_DEBUG.  A tool that
 *    serialises dispatch without any of these (e.g. a debugger attached after
 *    start-up) costs one timeout per call: set QPSK_PIPELINE_GATE=0 for such
 *    runs (results are identical with the gate off; only the overlap order may
 *    vary).
 *    QPSK_PIPELINE_GATE=1 forces it on.  Read once per handle, at create.
 */
int qpsk_demod_process_async(qpsk_demod *h, int32_t mode, const float *iq, int64_t stride_floats,
                             int64_t n_samples, const int64_t *lengths, uint8_t *bits,
                             int64_t bits_stride_bytes, int64_t *n_bits, float *syms,
                             int64_t syms_stride_floats, int64_t *n_syms);
/* 1 if handles created now use the residency gate, 0 if the environment turns
 * it off (the list above); needs no device. */
int qpsk_pipeline_gate_enabled(void);
/* Residency-gate waits of this handle that ran out (QPSK_GATE_TIMEOUT_MS) since
 * it was created, after every queued call; 0 in normal operation.  Besides
 * serialised dispatch, contention can also run a wait out: at most one loop
 * workgroup fits a CU (its LDS), so another handle's or process's loop kernel
 * holding every CU for longer than the cap delays this one's workgroups past
 * it.  Nothing hangs and no result changes; only the overlap order of that
 * call may differ.  Raise QPSK_GATE_TIMEOUT_MS where handles share a GPU with
 * long calls.  (QPSK_GATE_NO_PUBLISH=1 is a test hook that suppresses the
 * count so every wait runs out; it is honoured only together with
 * QPSK_PIPELINE_GATE=1.) */
int qpsk_demod_gate_timeouts(qpsk_demod *h, uint64_t *count);
/* The symbol-loop shape qpsk_demod_create picks for loop_variant = 0 (auto):
 * at sps >= 8, 7 (6 streams x 512-sample rounds) while ceil(S/6) <= cus, else
 * 6 (12 x 256) while ceil(S/12) <= cus, else 0 (the launcher's default for the
 * sps: 32 x 64 at sps >= 2).  (24 x 128, variant 4, needed ceil(S/24) <= cus/2,
 * which no batch past the 12 x 256 bound meets; it is only picked on request.)
 * A requested variant != 0 is returned unchanged.  Needs no device. */
int32_t qpsk_demod_pick_loop_variant(int32_t requested, int32_t n_streams, double sps, int32_t cus);
/* OR of the QPSK_STATUS_* flags raised since the last qpsk_demod_status call
 * (waits for every queued call), then cleared.  0 = every call so far stayed
 * inside the reference's defined behaviour. */
int qpsk_demod_status(qpsk_demod *h, uint32_t *flags);

/* The matched-filter output (ComplexFIRFilter.Filter, FIRFilter.cs:80-91) of
 * the last synchronous qpsk_demod_process call of at most max_samples_per_call
 * samples: n_samples per stream into out [S][stride_floats] (host or device
 * memory).  For inspection and FIR parity checks; pipelined and chunked calls
 * leave other buffers behind. */
int qpsk_demod_last_mf(qpsk_demod *h, float *out, int64_t stride_floats, int64_t n_samples, int32_t mem);

/* Make hip_stream wait for every pipelined call issued so far (NULL: block the
 * calling host thread until they are done). */
int qpsk_demod_pipeline_wait(qpsk_demod *h, void *hip_stream);
/* 2 = the stage boundary is double-buffered (front and back stages overlap),
 * 1 = no device memory was left for the second buffer (stages serialise),
 * 0 = no pipelined call yet. */
int qpsk_demod_pipeline_depth(const qpsk_demod *h);

/* Upper bounds a caller sizes outputs with, for a call of n_samples per stream. */
int64_t qpsk_demod_max_symbols(const qpsk_demod *h, int64_t n_samples);

/* First ordinal occurrence of tsc (a '0'/'1' string) in a packed bit row, i.e.
 * rx.IndexOf(_tsc, StringComparison.Ordinal) (QPSKDeModulator.cs:413-422).
 * Returns the bit index just past the TSC, or -1. */
int64_t qpsk_tsc_find(const uint8_t *bits, int64_t n_bits, const char *tsc);

/* Kernel launch times of the calls issued since timing was enabled (the first
 * 4096 of them), recorded by the kernels themselves: first workgroup start to
 * last workgroup end on the device's 100 MHz wall clock, so a launch's time is
 * its own span whichever stream or neighbour it ran beside (pipelined calls
 * included).  enable_timing(on) restarts the record.
 * stage_times: averages over the recorded calls of ms[0] = FLL, ms[1] =
 * matched-filter FIR, ms[2] = symbol-sync + Costas + decode kernel, ms[3] =
 * the call's kernel span (earliest start to latest end); a kernel that did not
 * run counts as absent.  Returns the number of entries written (<= 4).
 * launch_times: the same four values per call, ms[4*k .. 4*k+3] for call k
 * (0 = did not run); returns the number of calls written (<= max_calls).
 * kernel_clocks: per recorded call, the shader clock (GHz) the FLL, the FIR
 * and the loop kernel ran at, ghz[3*k .. 3*k+2]: shader-clock ticks
 * (s_memtime) over wall ticks of a sample of their waves' lifetimes (FIR:
 * every 64th workgroup; FLL: every workgroup; loop: every M&M wave; 0 = did
 * not run); returns the calls written. */
int qpsk_demod_enable_timing(qpsk_demod *h, int32_t on);
int qpsk_demod_stage_times(qpsk_demod *h, float *ms, int32_t n);
int qpsk_demod_launch_times(qpsk_demod *h, float *ms, int32_t max_calls);
int qpsk_demod_kernel_clocks(qpsk_demod *h, float *ghz, int32_t max_calls);

/* FIR phase sample (diagnostic): while on, every 64th matched-filter
 * workgroup adds the shader cycles of its three phases -- stage (HBM -> LDS),
 * products and sums, stores -- to one of two sums, chosen by whether a
 * symbol-loop workgroup of this handle held its CU when it started (each loop
 * workgroup marks its CU, read from the hardware HW_ID / XCC_ID registers).
 * fir_phases: out[8 * shared + k], k = 0 stage, 1 compute, 2 store cycles, 3
 * workgroups, shared = 0 free CU / 1 loop-shared CU (n >= 16); the sums are
 * then cleared.  Returns 16. */
int qpsk_demod_enable_fir_phases(qpsk_demod *h, int32_t on);
int qpsk_demod_fir_phases(qpsk_demod *h, uint64_t *out, int32_t n);

/* Design products, for parity checks against the reference constructor. */
int qpsk_demod_rrc_taps(const qpsk_demod *h, float *taps, int32_t cap);
int qpsk_demod_gains(const qpsk_demod *h, double *mm_sps, double *kp, double *ki,
                     double *costas_alpha, double *costas_beta);
int qpsk_demod_fll_taps(const qpsk_demod *h, float *lower_iq, float *upper_iq, int32_t cap_floats);

/* Constructor math without a device: RRC taps (float, as widened by
 * ToInterleavedIQRealTaps, QPSKDeModulator.cs:278-288), gains[5] = {M&M sps,
 * kp, ki, Costas alpha, Costas beta}, FLL band-edge taps (interleaved, 80
 * floats each).  Returns the tap count or an error (same validation as create). */
int qpsk_demod_design(const qpsk_demod_params *p, float *rrc_taps, int32_t cap, double *gains,
                      float *fll_lower_iq, float *fll_upper_iq);

/* Loop state snapshot (checkpoint / migration): a 32-byte header (magic
 * "QPSK", format 2, streams, RRC taps, carry length, FLL taps, record size)
 * then one record per stream, the M&M carries, FIR histories and FLL delay
 * lines.  get_state needs buf_bytes >= state_bytes; set_state needs exactly
 * state_bytes and a header matching this handle, else QPSK_ERR_ARGUMENT (a
 * blob of another handle shape or library version is never misread).  Both
 * first wait for (and flush) pipelined calls. */
int64_t qpsk_demod_state_bytes(const qpsk_demod *h);
int qpsk_demod_get_state(qpsk_demod *h, void *host_buf, int64_t buf_bytes);
int qpsk_demod_set_state(qpsk_demod *h, const void *host_buf, int64_t buf_bytes);

/* ---------------------------------------------------------------------------
 * Multi-GPU group: one batch of n_streams over several GPUs,
 * for a host (the C# shim, a C++ driver) that wants the whole node behind one
 * object.  Every reference instance owns its loop state (QPSKDeModulator.cs:20-73),
 * so the batch splits into contiguous shards with no exchange: shard k =
 * streams [n*k/n_dev, n*(k+1)/n_dev) on devices[k], one ordinary handle each
 * (the split bench.py's ranks use).  A group call slices the caller's rows by
 * row offset (shard k reads iq + first_k*stride_floats, lengths + first_k and
 * writes bits + first_k*bits_stride_bytes, n_bits + first_k, syms + ..., n_syms
 * + ...), runs every shard at once on its own worker thread, and returns when
 * all are done.  Results equal one handle's over the whole batch, stream for
 * stream.  One caller thread per group, as for a handle.
 */
typedef struct qpsk_demod_group qpsk_demod_group;
/* Contiguous shard k of n_parts over n_streams: *first = n_streams*k/n_parts,
 * *count = n_streams*(k+1)/n_parts - *first.  Needs no device. */
int qpsk_shard_streams(int32_t n_streams, int32_t n_parts, int32_t k, int32_t *first, int32_t *count);
/* n_dev handles with params p (p->device ignored: shard k lives on devices[k];
 * a device may repeat, e.g. two shards on device 0).  n_streams >= n_dev. */
int qpsk_demod_group_create(const qpsk_demod_params *p, const int32_t *devices, int32_t n_dev,
                            int32_t n_streams, qpsk_demod_group **out);
/* Waits for every shard's work, destroys the handles, stops the workers. */
int qpsk_demod_group_destroy(qpsk_demod_group *g);
/* Number of shards (n_dev). */
int qpsk_demod_group_size(const qpsk_demod_group *g);
/* Shard k's first stream, stream count, device and handle (any may be NULL).
 * The handle belongs to the group; use it for device-resident batches on a
 * multi-GPU group (pointers on that shard's device), streams, timing. */
int qpsk_demod_group_shard(const qpsk_demod_group *g, int32_t k, int32_t *first_stream, int32_t *n_streams,
                           int32_t *device, qpsk_demod **handle);
/* qpsk_demod_process on every shard, fanned out and joined; arguments as for
 * one handle over all n_streams rows.  mem = QPSK_MEM_HOST (the C# spans) on
 * any group; QPSK_MEM_DEVICE only when every shard is on one device (else
 * QPSK_ERR_ARGUMENT: call the shard handles), and the call then returns with
 * the outputs written (each shard's stream is joined).  Arguments are checked
 * on the whole batch before any shard runs; a shard that fails later returns
 * its status with "shard k (device d): ..." in qpsk_last_error, the other
 * shards' calls having run (as independent C# instances would). */
int qpsk_demod_group_process(qpsk_demod_group *g, int32_t mode, const float *iq, int64_t stride_floats,
                             int64_t n_samples, const int64_t *lengths, int32_t mem, uint8_t *bits,
                             int64_t bits_stride_bytes, int64_t *n_bits, float *syms, int64_t syms_stride_floats,
                             int64_t *n_syms);
/* Per-shard checkpoint / migration: qpsk_demod_state_bytes / get_state /
 * set_state of shard k's handle (0 bytes for a bad k). */
int64_t qpsk_demod_group_state_bytes(const qpsk_demod_group *g, int32_t k);
int qpsk_demod_group_get_state(qpsk_demod_group *g, int32_t k, void *host_buf, int64_t buf_bytes);
int qpsk_demod_group_set_state(qpsk_demod_group *g, int32_t k, const void *host_buf, int64_t buf_bytes);

/* ---------------------------------------------------------------------------
 * Host-fed streaming front-end: the deployment shape of
 * ModDemodOverSDR.cs:116-183, where the SDR thread hands CF32 buffers to
 * DeModulate one after another.  A ring of `depth` pinned host slots feeds one
 * handle: submit k uploads slot k on the DMA engine and queues a pipelined
 * DeModulate of it (qpsk_demod_process_async), so chunk k+1's upload overlaps
 * chunk k's matched filter and symbol loop, and chunk k's bits come back while
 * chunk k+1 computes.  collect returns the oldest outstanding chunk's bits.
 * Results equal consecutive qpsk_demod_process calls on the same chunks.  One
 * caller thread per ring, as for the handle (QPSKDeModulator is not
 * thread-safe either).
 */
typedef struct qpsk_rx qpsk_rx;
/* depth: 2..8 slots of n_streams x max_samples_per_call complex samples.  The
 * ring binds the handle to its own upload stream (as qpsk_demod_set_stream);
 * do not call the handle directly while the ring lives. */
int qpsk_rx_create(qpsk_demod *h, int32_t depth, qpsk_rx **out);
/* Waits for every outstanding chunk, then frees the ring (the handle keeps its
 * state and returns to a library-owned stream). */
int qpsk_rx_destroy(qpsk_rx *r);
/* The pinned host slot the next submit reads, [n_streams][*stride_floats]
 * interleaved I,Q: fill it in place (e.g. as an SDR driver's receive buffer)
 * and pass it to submit to skip the host copy.  QPSK_ERR_STATE while that slot
 * still holds an uncollected chunk. */
int qpsk_rx_next_slot(qpsk_rx *r, float **iq, int64_t *stride_floats);
/* Queue one DeModulate call on every stream.  iq: host rows, copied into the
 * slot unless iq is the slot itself; n_samples / lengths as in
 * qpsk_demod_process.  *ticket = the call's sequence number (may be NULL).
 * QPSK_ERR_STATE when all depth slots hold uncollected chunks. */
int qpsk_rx_submit(qpsk_rx *r, const float *iq, int64_t stride_floats, int64_t n_samples,
                   const int64_t *lengths, int64_t *ticket);
/* Wait for the oldest uncollected chunk and copy its bits (packed MSB-first,
 * as qpsk_demod_process) and bit counts to host memory.  QPSK_ERR_STATE when
 * nothing is outstanding. */
int qpsk_rx_collect(qpsk_rx *r, uint8_t *bits, int64_t bits_stride_bytes, int64_t *n_bits,
                    int64_t *ticket);

/* ---------------------------------------------------------------------------
 * Byte framer (DeModulateBytes, QPSKDeModulator.cs:169-259), batched: one
 * framer per stream fed with the packed bits of each process() call.
 */
typedef struct qpsk_framer qpsk_framer;
int qpsk_framer_create(int32_t n_streams, const uint8_t *start_marker, int32_t n_start,
                       const uint8_t *end_marker, int32_t n_end, int64_t ring_capacity,
                       qpsk_framer **out);
int qpsk_framer_destroy(qpsk_framer *f);
/* DeModulateBytes takes its markers per call; change them without touching
 * the framer state. */
int qpsk_framer_set_markers(qpsk_framer *f, const uint8_t *start_marker, int32_t n_start,
                            const uint8_t *end_marker, int32_t n_end);
/* Feed one call's (post-TSC) bits for every stream (host memory); payload[s]
 * receives the completed frame of this call if any (length in n_payload[s],
 * 0 = none), exactly like one DeModulateBytes return value. */
int qpsk_framer_push(qpsk_framer *f, const uint8_t *bits, int64_t bits_stride_bytes,
                     const int64_t *bit_offset, const int64_t *n_bits, uint8_t *payload,
                     int64_t payload_stride, int64_t *n_payload);

/* ---------------------------------------------------------------------------
 * Device-resident framer and TSC search: the same
 * DeModulateBytes state machine (QPSKDeModulator.cs:169-259) and TSC strip
 * (:413-422), one workgroup per stream, fed straight from process()'s device
 * bit rows with no host round trip.  Every pointer below is device memory and
 * every call is ordered on the framer's stream.  The ring is a per-stream
 * linear buffer of ring_capacity bytes (RingClear resets head to 0 and nothing
 * consumes from the tail, so the reference ring never wraps inside a frame);
 * overflow drops the frame and resyncs exactly like RingTryWriteByte (:95-103).
 */
typedef struct qpsk_framer_dev qpsk_framer_dev;
/* ring_capacity <= 0 selects the reference's 300_000_000 bytes per stream (:58). */
int qpsk_framer_dev_create(int32_t n_streams, const uint8_t *start_marker, int32_t n_start,
                           const uint8_t *end_marker, int32_t n_end, int64_t ring_capacity,
                           int32_t device, qpsk_framer_dev **out);
int qpsk_framer_dev_destroy(qpsk_framer_dev *f);
/* Bind to a caller-owned hipStream_t (NULL = library-owned stream). */
int qpsk_framer_dev_set_stream(qpsk_framer_dev *f, void *hip_stream);
/* Per-call markers (DeModulateBytes takes them per call); state is kept. */
int qpsk_framer_dev_set_markers(qpsk_framer_dev *f, const uint8_t *start_marker, int32_t n_start,
                                const uint8_t *end_marker, int32_t n_end);
/* One DeModulateBytes step on every stream: bits rows as qpsk_demod_process
 * wrote them, bit_offset[s] (NULL = 0) = first payload bit after the TSC, or
 * < 0 when this call's TSC search failed (DeModulate returned ""); payload[s]
 * receives the frame completed by this call (first payload_stride bytes) and
 * n_payload[s] its full length (0 = none). */
int qpsk_framer_dev_push(qpsk_framer_dev *f, const uint8_t *bits, int64_t bits_stride_bytes,
                         const int64_t *bit_offset, const int64_t *n_bits, uint8_t *payload,
                         int64_t payload_stride, int64_t *n_payload);
/* Host copy of every stream's framer status (arrays of n_streams, any may be
 * NULL; synchronises the framer's stream): in-frame flag, ring bytes held,
 * start-hunt carry bits. */
int qpsk_framer_dev_status(const qpsk_framer_dev *f, int32_t *in_frame, int64_t *ring_count,
                           int64_t *carry_bits);
/* qpsk_tsc_find for every stream of a device bit batch: offsets[s] = bit index
 * just past the first TSC occurrence in row s, -1 if absent, 0 for a NULL or
 * blank tsc.  Ordered on hip_stream (NULL = the null stream). */
int qpsk_tsc_find_device(const uint8_t *bits, int64_t bits_stride_bytes, const int64_t *n_bits,
                         int32_t n_streams, const char *tsc, int64_t *offsets, void *hip_stream);

/* ---------------------------------------------------------------------------
 * Synthetic batched input (QPSKModulator.Modulate + the test bench channel),
 * generated in device memory.  Stream s draws its payload from
 * splitmix64(seed ^ s); tx_bits receives the payload bits (packed MSB-first).
 * cfo_hz: per-stream carrier offset drawn U[-cfo_hz, +cfo_hz] (0 = clean
 * ±ppm LO pair), multipath: 4-tap channel [1, .25e^{j.7}, .1e^{-j1.9}, .05],
 * esn0_db: AWGN Es/N0 (>= 200 = none).  lo_ppm = cfo_hz = 0: no carrier at
 * all, i.e. QPSKModulator.Modulate's own baseband (QPSKModulator.cs:104-167).
 */
typedef struct qpsk_synth_params {
    int32_t sample_rate, symbol_rate;
    double rrc_alpha;
    int32_t rrc_span;
    int32_t differential;
    uint64_t seed;
    double lo_ppm;
    double cfo_hz;
    int32_t multipath;
    double esn0_db;
    int64_t first_stream;       /* global id of row 0: a rank's shard draws the same
                                   streams whatever the sharding */
    int32_t reserved[6];
} qpsk_synth_params;
void qpsk_synth_params_init(qpsk_synth_params *p, int32_t sample_rate, int32_t symbol_rate);
int qpsk_synth_generate(const qpsk_synth_params *p, int32_t device, void *hip_stream,
                        int32_t n_streams, int64_t n_samples, float *iq_dev,
                        int64_t stride_floats, uint8_t *tx_bits_dev, int64_t bits_stride_bytes);

/* ---------------------------------------------------------------------------
 * QPSKModulator (QPSKModulator.cs:18-167) behind the same ABI, batched: one
 * handle = one constructor (RRC taps, TSC, differential flag), one call =
 * Modulate (or ModulateBytes) on S independent bit strings, computed on the
 * GPU.  The impulse train (symbol d at delay + d*sps, delay = (T-1)/2) is
 * filtered by the float RRC taps in double and rounded to float, i.e.
 * fftFilter's output (FIRFilter.cs:96-141) restated as direct convolution;
 * output length = delay + nDibits*sps (+ delay when pulse shaping).
 * ModulateTextUtf8 (:74-89) is ModulateBytes on Encoding.GetBytes results and
 * stays in the C# shim.
 */
typedef struct qpsk_mod_params {
    int32_t sample_rate;        /* int SampleRate                 */
    int32_t symbol_rate;        /* int SymbolRate                 */
    double rrc_alpha;           /* double RrcAlpha = 0.9          */
    int32_t rrc_span;           /* int rrcSpan = 6                */
    int32_t differential;       /* bool differentialEncoding = true */
    int32_t device;             /* HIP device ordinal             */
    int32_t reserved[7];
} qpsk_mod_params;
typedef struct qpsk_mod qpsk_mod;
void qpsk_mod_params_init(qpsk_mod_params *p, int32_t sample_rate, int32_t symbol_rate);
/* new QPSKModulator(..., tsc): tsc is a '0'/'1' string prepended to every
 * Modulate call's data (NULL or blank = none, string.IsNullOrWhiteSpace). */
int qpsk_mod_create(const qpsk_mod_params *p, const char *tsc, qpsk_mod **out);
int qpsk_mod_destroy(qpsk_mod *m);
int qpsk_mod_set_stream(qpsk_mod *m, void *hip_stream);
/* floats one row of Modulate output holds for n_bits payload bits */
int64_t qpsk_mod_output_floats(const qpsk_mod *m, int64_t n_bits, int32_t pulse_shaping);
/* Modulate(string data, bool pulseShaping) on every stream: bits [S][stride]
 * packed MSB-first (bit i of the string = bit 7 - i%8 of byte i/8), n_bits[s]
 * bits each (an odd count drops the last bit, :113); out [S][out_stride]
 * interleaved float, n_out_floats[s] = its length (0 for < 2 bits in all).
 * mem applies to bits, n_bits, out and n_out_floats. */
int qpsk_mod_modulate(qpsk_mod *m, int32_t n_streams, const uint8_t *bits, int64_t bits_stride_bytes,
                      const int64_t *n_bits, int32_t pulse_shaping, int32_t mem, float *out,
                      int64_t out_stride_floats, int64_t *n_out_floats);
/* ModulateBytes(payload, startMarker, endMarker, pulseShaping) (:54-72) on every
 * stream, host memory: payload [S][payload_stride] bytes, n_payload[s] each.
 * Empty markers are QPSK_ERR_ARGUMENT (ArgumentException, :60-61). */
int qpsk_mod_modulate_bytes(qpsk_mod *m, int32_t n_streams, const uint8_t *payload, int64_t payload_stride,
                            const int64_t *n_payload, const uint8_t *start_marker, int32_t n_start,
                            const uint8_t *end_marker, int32_t n_end, int32_t pulse_shaping, float *out,
                            int64_t out_stride_floats, int64_t *n_out_floats);

const char *qpsk_last_error(void);
int qpsk_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
