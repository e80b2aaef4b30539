/*
 * c_abi_demo.c -- the drop-in boundary used from plain C (no Python, no torch,
 * no HIP headers): what a cgo / JNI / P/Invoke binding of include/qpsk_demod.h
 * does.  S streams of differential QPSK (oracle modulator, testAtDataLevel-like
 * sps 8 / 65 taps / alpha 0.4, each stream with its own LO pair) go through
 *   1. qpsk_demod_process on host memory, in ragged chunks,
 *   2. the host-fed ring (qpsk_rx_*) on a second handle, and
 *   3. a multi-GPU group (qpsk_demod_group_*: the C++ multi-GPU driver's
 *      entry) over the devices in QPSK_DEMO_DEVICES
 *      (comma list, default "0,0": two shards on device 0),
 * and every call's bits must equal the oracle's DeModulate on the same chunk
 * (or_demod_demodulate_ex, QPSKDeModulator.cs:345-410; test infrastructure).
 * Exit status 0 = identical.  Built by tools/c_abi_demo.mk (build());
 * run by tests/test_gpu_parity.py::test_c_abi_demo_from_plain_c.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "qpsk_demod.h"
#include "qpsk_oracle.h"

#define S 4
#define CALLS 5
#define FS 10000000
#define RS 1250000

static uint64_t sm(uint64_t *x) {   /* splitmix64 */
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int check(int rc, const char *what) {
    if (rc < 0) {
        fprintf(stderr, "%s failed: %d %s\n", what, rc, qpsk_last_error());
        exit(2);
    }
    return rc;
}

/* MSB-first packed bits (BitPacker order) vs the oracle's '0'/'1' string */
static int same_bits(const uint8_t *row, int64_t nb, const char *ref, long nref) {
    if (nb != nref) return 0;
    for (int64_t i = 0; i < nb; ++i)
        if (((row[i >> 3] >> (7 - (i & 7))) & 1) != (ref[i] - '0')) return 0;
    return 1;
}

int main(void) {
    const int nbits = 6000;
    long nf[S];
    float *sig[S];
    for (int s = 0; s < S; ++s) {
        uint64_t seed = 0x5159534Bull ^ (uint64_t)s;
        char *bits = malloc(nbits + 1);
        for (int i = 0; i < nbits; ++i) bits[i] = (char)('0' + (sm(&seed) & 1));
        bits[nbits] = 0;
        const long cap = 2L * (nbits / 2) * (FS / RS) + 65536;
        sig[s] = malloc(cap * sizeof(float));
        nf[s] = or_modulate(FS, RS, 0.4f, 8, 1, NULL, bits, nbits, 1, sig[s], cap);
        or_nco *tx = or_nco_new(100e6, FS, 1.0, 0.0, 0x1000 + s);
        or_nco *rx = or_nco_new(100e6, FS, -1.0, 0.0, 0x2000 + s);
        or_apply_lo_pair(tx, rx, sig[s], nf[s] / 2);
        or_nco_free(tx);
        or_nco_free(rx);
        free(bits);
    }
    long n_min = nf[0] / 2;
    for (int s = 1; s < S; ++s) n_min = nf[s] / 2 < n_min ? nf[s] / 2 : n_min;

    /* ragged per-stream chunk lengths: call c of stream s covers [pos, pos + len) */
    int64_t len[CALLS][S], pos[CALLS][S];
    uint64_t rs = 7;
    for (int s = 0; s < S; ++s) {
        int64_t p = 0;
        for (int c = 0; c < CALLS; ++c) {
            int64_t l = c == CALLS - 1 ? n_min - p : (int64_t)(sm(&rs) % (uint64_t)(n_min / CALLS)) + 1;
            if (c == 2 && s == 1) l = 0;                  /* an empty call (QPSKDeModulator.cs:350-351) */
            pos[c][s] = p;
            len[c][s] = l;
            p += l;
        }
    }
    int64_t n_call_max = 0;
    for (int c = 0; c < CALLS; ++c)
        for (int s = 0; s < S; ++s) n_call_max = len[c][s] > n_call_max ? len[c][s] : n_call_max;

    qpsk_demod_params p;
    qpsk_demod_params_init(&p, FS, RS);
    p.rrc_alpha = 0.4f;
    p.rrc_span = 8;
    p.max_samples_per_call = n_call_max;
    qpsk_demod *h, *h2;
    check(qpsk_demod_create(&p, S, &h), "create");
    check(qpsk_demod_create(&p, S, &h2), "create (ring)");
    qpsk_rx *ring;
    check(qpsk_rx_create(h2, 2, &ring), "rx_create");
    int32_t devs[8];
    int n_dev = 0;
    {
        const char *e = getenv("QPSK_DEMO_DEVICES");
        char buf[64];
        snprintf(buf, sizeof buf, "%s", e && *e ? e : "0,0");
        for (char *t = strtok(buf, ","); t && n_dev < 8; t = strtok(NULL, ",")) devs[n_dev++] = atoi(t);
    }
    qpsk_demod_group *grp;
    check(qpsk_demod_group_create(&p, devs, n_dev, S, &grp), "group_create");
    for (int k = 0; k < n_dev; ++k) {
        int32_t f, c, d;
        check(qpsk_demod_group_shard(grp, k, &f, &c, &d, NULL), "group_shard");
        int32_t f2, c2;
        check(qpsk_shard_streams(S, n_dev, k, &f2, &c2), "shard_streams");
        if (f != f2 || c != c2 || d != devs[k]) {
            fprintf(stderr, "shard %d: [%d, +%d) on %d, expected [%d, +%d) on %d\n", k, f, c, d, f2, c2, devs[k]);
            return 1;
        }
    }

    const int64_t stride = 2 * n_call_max;
    const int64_t bstride = (2 * qpsk_demod_max_symbols(h, n_call_max) + 7) / 8 + 8;
    float *iq = calloc((size_t)S * stride, sizeof(float));
    uint8_t *bits = calloc((size_t)S * bstride, 1), *bits2 = calloc((size_t)S * bstride, 1);
    uint8_t *bits3 = calloc((size_t)S * bstride, 1);
    int64_t nb[S], nb2[S], nb3[S];
    or_demod *ref[S];
    for (int s = 0; s < S; ++s) {
        or_demod_cfg cfg;
        or_demod_cfg_default(&cfg, FS, RS);
        cfg.rrc_alpha = 0.4f;
        cfg.rrc_span = 8;
        int err = 0;
        ref[s] = or_demod_new(&cfg, &err);
    }
    char *rb = malloc((size_t)n_call_max * 2 + 16);
    float *rsym = malloc(((size_t)n_call_max * 2 + 16) * sizeof(float));
    int bad = 0;
    for (int c = 0; c < CALLS; ++c) {
        for (int s = 0; s < S; ++s)
            memcpy(iq + s * stride, sig[s] + 2 * pos[c][s], (size_t)(2 * len[c][s]) * sizeof(float));
        check(qpsk_demod_process(h, QPSK_MODE_DEMODULATE, iq, stride, 0, len[c], QPSK_MEM_HOST, bits, bstride, nb,
                                 NULL, 0, NULL), "process");
        check(qpsk_rx_submit(ring, iq, stride, 0, len[c], NULL), "rx_submit");
        check(qpsk_rx_collect(ring, bits2, bstride, nb2, NULL), "rx_collect");
        check(qpsk_demod_group_process(grp, QPSK_MODE_DEMODULATE, iq, stride, 0, len[c], QPSK_MEM_HOST, bits3,
                                       bstride, nb3, NULL, 0, NULL), "group_process");
        for (int s = 0; s < S; ++s) {
            long nsy = 0, tsc = 0;
            const long nr = or_demod_demodulate_ex(ref[s], sig[s] + 2 * pos[c][s], 2 * len[c][s], rb,
                                                   n_call_max * 2 + 16, rsym, n_call_max * 2 + 16, &nsy, &tsc);
            if (!same_bits(bits + s * bstride, nb[s], rb, nr)) {
                fprintf(stderr, "call %d stream %d: process() bits differ (%lld vs %ld)\n", c, s, (long long)nb[s], nr);
                bad = 1;
            }
            if (!same_bits(bits2 + s * bstride, nb2[s], rb, nr)) {
                fprintf(stderr, "call %d stream %d: ring bits differ (%lld vs %ld)\n", c, s, (long long)nb2[s], nr);
                bad = 1;
            }
            if (!same_bits(bits3 + s * bstride, nb3[s], rb, nr)) {
                fprintf(stderr, "call %d stream %d: group bits differ (%lld vs %ld)\n", c, s, (long long)nb3[s], nr);
                bad = 1;
            }
        }
    }
    check(qpsk_rx_destroy(ring), "rx_destroy");
    check(qpsk_demod_group_destroy(grp), "group_destroy");
    check(qpsk_demod_destroy(h2), "destroy");
    check(qpsk_demod_destroy(h), "destroy");
    for (int s = 0; s < S; ++s) {
        or_demod_free(ref[s]);
        free(sig[s]);
    }
    free(iq); free(bits); free(bits2); free(bits3); free(rb); free(rsym);
    printf("c_abi_demo: %d streams x %d ragged calls (%lld samples), process(), qpsk_rx and a %d-shard group: %s\n",
           S, CALLS, (long long)n_min, n_dev, bad ? "MISMATCH" : "bits identical to the oracle");
    return bad;
}
