/* check_glibc_sin.c -- the glibc double sin/cos restatement (oracle copy,
 * oracle/or_glibc_trig.h; the product copy is pinned equal to it by
 * tests/test_oracle.py) against this host's real libm sin and cos.
 *
 *   gcc -O2 -ffp-contract=off -Ioracle tools/check_glibc_sin.c -o tools/bin/check_glibc_sin -lm
 *   (add -DWITH_PRODUCT -Iqpsk-modulator-demodulator_amd/csrc to check the product copy as well)
 *   tools/bin/check_glibc_sin [scale]     (scale multiplies every sample count)
 *
 * Samples: uniform in [-8, 8] (the Costas phase and all five argument
 * regions), uniform in [-2^27, 2^27] (the three-part pi/2 reduction), random
 * bit patterns of every exponent, [1e8, 1e300] (Payne-Hanek), and sweeps of
 * +-4096 ulps around every region threshold, 0.126, multiples of pi/4 and the
 * table's rounding points (i + 1/2)/128.  Exit status 1 on any difference
 * (NaN compares equal to NaN). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "or_glibc_trig.h"
#ifdef WITH_PRODUCT
/* the product copy too: -DWITH_PRODUCT -Iqpsk-modulator-demodulator_amd/csrc */
#include "qpsk_glibc_trig.h"
#endif

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next64(void)
{
    uint64_t z = (rng += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double uni(double lo, double hi) { return lo + (hi - lo) * ((next64() >> 11) * 0x1p-53); }

static long n_checked, n_bad;
#ifdef WITH_PRODUCT
static double g_tabs[440], g_tabc[440];   /* the split form's two table layouts */
#endif
static double (*volatile libm_sin)(double) = sin;
static double (*volatile libm_cos)(double) = cos;

static int same(double a, double b)
{
    if (a != a && b != b) return 1;
    return or_gl_bits(a) == or_gl_bits(b);
}

static void check(double x)
{
    const double s = or_glibc_sin(x), c = or_glibc_cos(x);
    const double rs = libm_sin(x), rc = libm_cos(x);
    ++n_checked;
#ifdef WITH_PRODUCT
    const double ps = qpsk_glibc_sin(x, qpsk_gl_sincostab_host), pc = qpsk_glibc_cos(x, qpsk_gl_sincostab_host);
    if (!same(ps, s) || !same(pc, c)) {
        if (n_bad < 20) printf("x=%a product sin %a cos %a vs oracle %a %a\n", x, ps, pc, s, c);
        ++n_bad;
    }
    double bs, bc;   /* the branch-free form */
    qpsk_glibc_sincos_bf(x, qpsk_gl_sincostab_host, &bs, &bc);
    if (!same(bs, s) || !same(bc, c)) {
        if (n_bad < 20) printf("x=%a branch-free sin %a cos %a vs oracle %a %a\n", x, bs, bc, s, c);
        ++n_bad;
    }
    double ss, sc;   /* the split form the GPU Costas loop runs (two lanes per argument) */
    qpsk_glibc_sincos_split_host(x, g_tabs, g_tabc, &ss, &sc);
    if (!same(ss, s) || !same(sc, c)) {
        if (n_bad < 20) printf("x=%a split sin %a cos %a vs oracle %a %a\n", x, ss, sc, s, c);
        ++n_bad;
    }
    if (!(fabs(x) >= QPSK_GLIBC_SMALL_LIMIT)) {   /* the fast split pair (its range, NaN included) */
        double fs, fc;
        qpsk_glibc_sincos_fs_host(x, g_tabs, g_tabc, &fs, &fc);
        if (!same(fs, s) || !same(fc, c)) {
            if (n_bad < 20) printf("x=%a fast split sin %a cos %a vs oracle %a %a\n", x, fs, fc, s, c);
            ++n_bad;
        }
    }
#endif
    if (!same(s, rs) || !same(c, rc)) {
        if (n_bad < 20)
            printf("x=%a sin %a vs libm %a   cos %a vs libm %a\n", x, s, rs, c, rc);
        ++n_bad;
    }
}

static void sweep(double x, int ulps)
{
    for (int s = -1; s <= 1; s += 2) {
        double y = s * x;
        for (int i = 0; i < ulps; ++i) {
            check(y);
            y = nextafter(y, s * INFINITY);
        }
        y = s * x;
        for (int i = 0; i < ulps; ++i) {
            y = nextafter(y, 0.0);
            check(y);
        }
    }
}

int main(int argc, char **argv)
{
    const long scale = argc > 1 ? atol(argv[1]) : 1;
#ifdef WITH_PRODUCT
    for (int i = 0; i < 110; ++i) qpsk_gl_half_tables(qpsk_gl_sincostab_host, i, g_tabs + 4 * i, g_tabc + 4 * i);
#endif
    for (long i = 0; i < scale * (1L << 24); ++i) check(uni(-8.0, 8.0));
    printf("[-8, 8]: %ld checked, %ld differ\n", n_checked, n_bad);
    for (long i = 0; i < scale * (1L << 22); ++i) check(uni(-0x1p27, 0x1p27));
    for (long i = 0; i < scale * (1L << 22); ++i) check(uni(-1.0, 1.0) * exp2(uni(-40.0, 0.0)));
    printf("+ [-2^27, 2^27] and small: %ld checked, %ld differ\n", n_checked, n_bad);
    for (long i = 0; i < scale * (1L << 21); ++i) {
        const double x = or_gl_from_bits(next64());
        if (isfinite(x)) check(x);
    }
    for (long i = 0; i < scale * (1L << 20); ++i) check((next64() & 1 ? -1.0 : 1.0) * exp2(uni(26.7, 996.0)));
    printf("+ random bits and Payne-Hanek: %ld checked, %ld differ\n", n_checked, n_bad);
    const uint32_t hi[] = {0x3e400000u, 0x3e500000u, 0x3feb6000u, 0x400368fdu, 0x419921fbu, 0x7fe00000u};
    for (unsigned j = 0; j < sizeof hi / sizeof hi[0]; ++j) sweep(or_gl_from_bits((uint64_t)hi[j] << 32), 4096);
    sweep(0.126, 4096);
    for (int q = 1; q < 64; ++q) sweep(q * 0.78539816339744830962, 4096);
    for (int i = 0; i < 110; ++i) sweep((i + 0.5) / 128.0, 256);
    check(0.0); check(-0.0); check(INFINITY); check(-INFINITY); check(NAN);
    check(0x1p-1074); check(-0x1p-1074); check(0x1.fffffffffffffp1023);
    printf("+ threshold sweeps: %ld checked, %ld differ\n", n_checked, n_bad);
    return n_bad ? 1 : 0;
}
